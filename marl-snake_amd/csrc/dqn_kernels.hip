// dqn_kernels.hip -- the fused consumer of the observations (SURVEY.md 8(f)
// rank 4): the reference's DQN forward (train_dqn.py:104-151, train_ga.py:60-
// 100) on the NHWC uint8 observation batch, on the bf16 matrix cores of gfx950.
//
//   x = obs (B, h, w, c) uint8 -> permute to NCHW, float (values 0/1: the
//       reference's x/255 branch is not taken, train_dqn.py:122)
//   conv1 c->32, conv2 32->64, conv3 64->64 (3x3, pad 1) + ReLU
//   flatten NCHW (index ch*h*w + y*w + x) -> fc1 (64hw->256) + ReLU
//   -> fc2 (256->128) + ReLU (= forward_features) -> fc3 (128->A)
//
// Two kernels:
//   k_dqn_conv  one wave per observation (many per CU): the three convolutions
//               as implicit GEMMs on v_mfma_f32_16x16x32_bf16, rows = the h*w
//               positions (padded to 16), columns = output channels, K = 9 taps
//               x input channels; the A fragments gathered from the previous
//               layer's NHWC bf16 image in the wave's LDS (8 consecutive k =
//               8 channels of one tap = one 16-byte read), the B fragments (the
//               weights, [cout][k] bf16) from global memory. conv3's ReLU output
//               goes to the scratch buffer as bf16 [B][64][P16] (NCHW, positions
//               padded to P16, the pad columns meet zero fc1 weights).
//   k_dqn_fc    128 observations per workgroup (8 waves x 16): fc1 as a GEMM
//               [128 x 64*P16] x [64*P16 x 256], the fc1 weight tile of each
//               32-wide k step staged once in LDS for all 8 waves (double
//               buffered); then per wave fc2 on the matrix cores (h1 from LDS)
//               and fc3 in fp32 on the vector units.
// Accumulation is fp32 everywhere; inputs and weights of the matrix products
// are bf16 (tolerance against the fp32 reference: tests/test_dqn.py).
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include "snake_internal.h"

namespace snake {
namespace dqn {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kFcObs = 256;       // observations per k_dqn_fc workgroup

__device__ __forceinline__ uint32_t bf16_bits(float x)   // round to nearest even
{
    const uint32_t u = __float_as_uint(x);
    return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}

__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// ---- k_dqn_conv ---------------------------------------------------------
// A workgroup of two waves runs one observation at a time through the three
// convolutions. Each layer's image lives in LDS as bf16 with a zero border
// ((h+2) x (w+2) positions q), chunk-major: 8 channels of one position = one
// 16-byte cell at chunk * R*16 + q*16 (R = positions rounded up to 16). The A
// fragment of tap (dy, dx) at GEMM row i is then one 16-byte read at a fixed
// offset from the row's own cell: no bounds checks, and with h, w and the
// channel counts compile-time the offset is an immediate. GEMM rows are
// assigned to positions so that the 16 rows of a tile have distinct q mod 16
// (row r of tile t = the t-th position with q % 16 == r): the lanes of every
// ds_read_b128 lane group then hit distinct banks for every tap. Each wave
// computes half the output channels (B fragments = weights, read from global
// memory through L1/L2 by every workgroup) for all row tiles, so each A
// fragment feeds NTW MFMAs.
__host__ __device__ constexpr int dqn_bidx(int p, int W) { return (p / W + 1) * (W + 2) + p % W + 1; }

// GEMM row (tile * 16 + q % 16) of observation position p
__host__ __device__ constexpr int dqn_row_of(int p, int W)
{
    const int r = dqn_bidx(p, W) & 15;
    int t = 0;
    for (int p2 = 0; p2 < p; p2++) t += (dqn_bidx(p2, W) & 15) == r;
    return t * 16 + r;
}

__host__ __device__ constexpr int dqn_tiles(int W)
{
    int mt = (W * W + 15) / 16;
    for (int p = 0; p < W * W; p++) {
        const int t = dqn_row_of(p, W) / 16 + 1;
        mt = t > mt ? t : mt;
    }
    return mt;
}

template <int VR, int CL>
struct Geo {
    static constexpr int W = 2 * VR + 1, H = W, P = H * W;
    static constexpr int MT = dqn_tiles(W), P16 = MT * 16;
    static constexpr int BW = W + 2, NB = BW * (H + 2);
    static constexpr int CP = 1 << CL;
    static constexpr int CH = ((NB + 15) / 16) * 16 * 16;       // bytes per 8-channel chunk plane
    static constexpr int K1S = (9 * CP + 31) / 32;              // conv1 k steps
    static constexpr int OFF1 = 0;                              // a1: 4 planes
    static constexpr int OFF2 = 4 * CH;                         // a2: 8 planes
    // a0 (CP/8 planes) in its own planes when four workgroups per CU still fit
    // (then no barrier closes an observation and a2's border is zeroed once),
    // else over a2 (its border rewritten after conv1 of every observation)
    static constexpr bool SEP = 4 * ((12 + CP / 8) * CH + P16 * 2) <= 160 * 1024;
    static constexpr int OFF0 = SEP ? 12 * CH : OFF2;
    static constexpr int OFFT = SEP ? 12 * CH + (CP / 8) * CH : 12 * CH;   // u16 [P16]: border index of GEMM row
    static constexpr int LDS = OFFT + P16 * 2;
    static constexpr int NCELL0 = NB * CP / 8;                  // 16-byte cells of the input image
    static constexpr int NBORDER = NB - P;
    __host__ __device__ static constexpr int tapoff(int tap) { return ((tap / 3) * BW + tap % 3) * 16; }
    // gather position of a padding row with q % 16 == r (finite values, results unused)
    __host__ __device__ static constexpr int padq(int r)
    {
        for (int q = BW + 1; q < NB - BW - 1; q++)
            if ((q & 15) == r) return q;
        return (H / 2 + 1) * BW + W / 2 + 1;
    }
};

__device__ __forceinline__ uint32_t pack2(float lo, float hi)
{
    return bf16_bits(lo) | (bf16_bits(hi) << 16);
}

// 8 bytes (0..255 each) -> 8 bf16 (exact; the conversions are v_cvt_f32_ubyteN)
__device__ __forceinline__ uint32_t bytes2_to_bf16(uint32_t v, int sh)
{
    return (__float_as_uint((float)((v >> sh) & 0xffu)) >> 16) |
           (__float_as_uint((float)((v >> (sh + 8)) & 0xffu)) & 0xffff0000u);
}

__device__ __forceinline__ u32x4 bytes_to_bf16(uint2 v)
{
    u32x4 r;
    r[0] = bytes2_to_bf16(v.x, 0);
    r[1] = bytes2_to_bf16(v.x, 16);
    r[2] = bytes2_to_bf16(v.y, 0);
    r[3] = bytes2_to_bf16(v.y, 16);
    return r;
}

// One 3x3 convolution of the workgroup's observation, this wave's NTW output
// channel tiles starting at tile nt0, from the chunk-major image at src.
// gpos[m] = byte offset of the lane's row cell minus one row and one column,
// plus the lane's chunk (quad) plane. Tap offsets per k step: compile-time for
// CIN >= 32 (one tap per k step), else the lane's precomputed toff[ks] (conv1
// with CIN < 32: chunk included, the quad plane taken back out).
template <int VR, int CL, int CIN, int KS, int NTW, int COUT, int MTW>
__device__ __forceinline__ void conv_mma(const uint8_t *lds, int src, const int *gpos, const int *toff,
                                         const uint16_t *__restrict__ wt, int nt0, int lane,
                                         f32x4 (&acc)[MTW][NTW])
{
    using G = Geo<VR, CL>;
    constexpr int K = KS * 32;
    // weights in fragment order (1 KB per (channel tile, k step), lane-major:
    // every load is 1 KB contiguous) through a buffer descriptor: the lane's
    // offset in one VGPR, the (tile, k step) part a scalar offset
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(wt), 0, 2 * K * COUT, 0x00020000);
    const int voff = 16 * lane;
    auto load_b = [&](bf16x8 (&bw)[NTW], int ks) {
#pragma unroll
        for (int j = 0; j < NTW; j++) {
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, 1024 * ((nt0 + j) * KS + ks), 0);
            bw[j] = __builtin_bit_cast(bf16x8, v);
        }
    };
#pragma unroll
    for (int m = 0; m < MTW; m++)
#pragma unroll
        for (int j = 0; j < NTW; j++) acc[m][j] = (f32x4)0.0f;
    auto a_off = [&](int ks) {
        if constexpr (CIN >= 32) return G::tapoff((ks * 32) / CIN) + ((ks * 32) % CIN) / 8 * G::CH;
        else return toff[ks];
    };
    // B and A (the row tiles' fragments of a k step) one k step ahead
    constexpr int ABUF = 2;
    // B fragments PF k steps ahead (2 and 3 measured no faster)
    constexpr int PF = 1, NR = PF + 1;
    bf16x8 bring[NR][NTW];
    bf16x8 abuf[ABUF][MTW];
#pragma unroll
    for (int i = 0; i < PF && i < KS; i++) load_b(bring[i], i);
    if constexpr (ABUF == 2) {
#pragma unroll
        for (int m = 0; m < MTW; m++) abuf[0][m] = *reinterpret_cast<const bf16x8 *>(lds + src + gpos[m] + a_off(0));
    }
#pragma unroll
    for (int ks = 0; ks < KS; ks++) {
        if (ks + PF < KS) load_b(bring[(ks + PF) % NR], ks + PF);
        // keep the prefetch ahead of this k step's MFMAs (the scheduler otherwise
        // sinks it next to its use: 4.78 -> 4.61 ms with the pin at 4 waves)
        __builtin_amdgcn_sched_barrier(0);
        bf16x8 *av = abuf[ABUF == 2 ? (ks & 1) : 0];
        if constexpr (ABUF == 2) {
            if (ks + 1 < KS) {
#pragma unroll
                for (int m = 0; m < MTW; m++)
                    abuf[(ks + 1) & 1][m] = *reinterpret_cast<const bf16x8 *>(lds + src + gpos[m] + a_off(ks + 1));
            }
        } else {
#pragma unroll
            for (int m = 0; m < MTW; m++) av[m] = *reinterpret_cast<const bf16x8 *>(lds + src + gpos[m] + a_off(ks));
        }
        const bf16x8 *bcur = bring[ks % NR];
#pragma unroll
        for (int m = 0; m < MTW; m++) {
#pragma unroll
            for (int j = 0; j < NTW; j++) acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[m], bcur[j], acc[m][j], 0, 0, 0);
        }
    }
}

// bias + ReLU -> bf16 into the interior of a chunk-major border image
template <int VR, int CL, int NTW, int MTW>
__device__ __forceinline__ void conv_store_lds(uint8_t *lds, int dst, const uint16_t *ptab, int nt0, int lane,
                                               const float (&bias)[NTW], f32x4 (&acc)[MTW][NTW])
{
    using G = Geo<VR, CL>;
    const int r16 = lane & 15, quad = lane >> 4;
#pragma unroll
    for (int j = 0; j < NTW; j++) {
        const int co = (nt0 + j) * 16 + r16;
        const float bb = bias[j];
        const int cbase = dst + (co >> 3) * G::CH + 2 * (co & 7);
#pragma unroll
        for (int m = 0; m < MTW; m++) {
            const uint2 pq = *reinterpret_cast<const uint2 *>(ptab + m * 16 + 4 * quad);
            const uint32_t q[4] = {pq.x & 0xffffu, pq.x >> 16, pq.y & 0xffffu, pq.y >> 16};
#pragma unroll
            for (int r = 0; r < 4; r++) {
                if (q[r] != 0xffffu)
                    *reinterpret_cast<uint16_t *>(lds + cbase + q[r] * 16) =
                        (uint16_t)bf16_bits(fmaxf(acc[m][j][r] + bb, 0.0f));
            }
        }
    }
}

struct ConvArgs {
    const uint8_t *obs;
    int64_t B;
    int C;                              // input channels (multiple of 8, <= CP)
    const uint16_t *w1, *w2, *w3;
    const float *b1, *b2, *b3;
    uint16_t *act;                      // [B][64 * P16], k order: snake_dqn_layout.fc1_w
};

template <int NW>
__device__ __forceinline__ void conv_sync()
{
    if constexpr (NW == 1) wave_lds_sync();
    else __syncthreads();
}

// NW waves per observation (1: no workgroup barriers, all four channel tiles of
// conv2/conv3 per wave, each A fragment feeding four MFMAs; 2: two waves split
// the channel tiles; 4: two channel halves x two row halves, for twice the
// waves per SIMD at the same LDS, each weight fragment loaded by two waves).
// ptab is passed to the epilogue offset to the wave's first row tile.
template <int VR, int CL, int NW>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(NW))) k_dqn_conv(const ConvArgs a)
{
    using G = Geo<VR, CL>;
    constexpr int NT = 64 * NW;
    constexpr int MH = NW == 4 ? 2 : 1, NH = NW == 1 ? 1 : 2;   // row-tile halves x channel halves
    constexpr int MTW = G::MT / MH;
    static_assert(G::MT % MH == 0, "row halves need an even tile count");
    constexpr int NC = (G::NCELL0 + NT - 1) / NT;
    __shared__ __attribute__((aligned(16))) uint8_t lds[G::LDS];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = NW == 1 ? 0 : __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform
    const int w = NH == 1 ? 0 : (wv & 1), m0 = MH == 1 ? 0 : (wv >> 1) * MTW;   // channel half, first row tile
    const int r16 = lane & 15;
    uint16_t *ptab = reinterpret_cast<uint16_t *>(lds + G::OFFT);
    for (int i = tid; i < G::P16; i += NT) ptab[i] = (uint16_t)0xffffu;
    // zero a1 (and a2 when the input image has its own planes): borders stay zero
    for (int i = tid; i < (G::SEP ? 12 : 4) * G::CH / 16; i += NT) reinterpret_cast<u32x4 *>(lds + G::OFF1)[i] = (u32x4)0u;
    conv_sync<NW>();
    for (int p = tid; p < G::P; p += NT) ptab[dqn_row_of(p, G::W)] = (uint16_t)dqn_bidx(p, G::W);
    conv_sync<NW>();
    const int qplane = (lane >> 4) * G::CH;
    int gpos[MTW];
#pragma unroll
    for (int m = 0; m < MTW; m++) {
        const int q = ptab[(m0 + m) * 16 + r16];
        gpos[m] = ((q != 0xffff ? q : G::padq(r16)) - G::BW - 1) * 16 + qplane;
    }
    // conv1 per-lane tap offsets (k = tap * CP + channel; taps past the 9th meet zero weights)
    int toff1[G::K1S];
#pragma unroll
    for (int ks = 0; ks < G::K1S; ks++) {
        const int k0 = ks * 32 + 8 * (lane >> 4), tap = k0 >> CL, ci = k0 & (G::CP - 1);
        toff1[ks] = (tap < 9 ? G::tapoff(tap) : G::tapoff(4)) + (ci >> 3) * G::CH - qplane;
    }
    // input cells of this thread (cell c: chunk c / NB, position c % NB): source
    // byte offset within the observation, or -1 (zero)
    int csrc[NC], cdst[NC];
#pragma unroll
    for (int i = 0; i < NC; i++) {
        const int c = tid + NT * i;
        const int g = c / G::NB, q = c % G::NB;
        const int y = q / G::BW - 1, x = q % G::BW - 1;
        const bool in = c < G::NCELL0 && (unsigned)y < (unsigned)G::H && (unsigned)x < (unsigned)G::W && g * 8 < a.C;
        csrc[i] = in ? (y * G::W + x) * a.C + g * 8 : -1;
        cdst[i] = c < G::NCELL0 ? G::OFF0 + g * G::CH + q * 16 : -1;
    }
    uint2 xin[NC];
    auto load_obs = [&](int64_t b) {
        const uint8_t *x = a.obs + b * (int64_t)(G::P * a.C);
#pragma unroll
        for (int i = 0; i < NC; i++) xin[i] = csrc[i] >= 0 ? *reinterpret_cast<const uint2 *>(x + csrc[i]) : make_uint2(0, 0);
    };
    constexpr int NT1 = 2 / NH, NT3 = 4 / NH;
    // biases of this lane's output channels, loaded once
    float bias1[NT1], bias2[NT3], bias3[NT3];
#pragma unroll
    for (int j = 0; j < NT1; j++) bias1[j] = a.b1[(w * NT1 + j) * 16 + r16];
#pragma unroll
    for (int j = 0; j < NT3; j++) {
        bias2[j] = a.b2[(w * NT3 + j) * 16 + r16];
        bias3[j] = a.b3[(w * NT3 + j) * 16 + r16];
    }
    int64_t b = blockIdx.x;
    if (b < a.B) load_obs(b);
    for (; b < a.B; b += gridDim.x) {
        // input image (whole, border included) over the a2 area
#pragma unroll
        for (int i = 0; i < NC; i++)
            if (cdst[i] >= 0) *reinterpret_cast<u32x4 *>(lds + cdst[i]) = bytes_to_bf16(xin[i]);
        if (b + gridDim.x < a.B) load_obs(b + gridDim.x);
        conv_sync<NW>();
        {   // conv1: CP -> 32
            f32x4 acc[MTW][NT1];
            conv_mma<VR, CL, G::CP, G::K1S, NT1, 32>(lds, G::OFF0, gpos, toff1, a.w1, w * NT1, lane, acc);
            conv_store_lds<VR, CL, NT1>(lds, G::OFF1, ptab + m0 * 16, w * NT1, lane, bias1, acc);
        }
        conv_sync<NW>();
        // the input image is dead: restore a2's zero border (overlaid case)
        if constexpr (!G::SEP) for (int i = tid; i < G::NBORDER * 8; i += NT) {
            const int bi = i >> 3, chunk = i & 7;
            int q;
            if (bi < G::BW) q = bi;
            else if (bi < 2 * G::BW) q = (G::H + 1) * G::BW + bi - G::BW;
            else q = (1 + ((bi - 2 * G::BW) >> 1)) * G::BW + ((bi - 2 * G::BW) & 1) * (G::BW - 1);
            *reinterpret_cast<u32x4 *>(lds + G::OFF2 + chunk * G::CH + q * 16) = (u32x4)0u;
        }
        {   // conv2: 32 -> 64
            f32x4 acc[MTW][NT3];
            conv_mma<VR, CL, 32, 9, NT3, 64>(lds, G::OFF1, gpos, nullptr, a.w2, w * NT3, lane, acc);
            conv_store_lds<VR, CL, NT3>(lds, G::OFF2, ptab + m0 * 16, w * NT3, lane, bias2, acc);
        }
        conv_sync<NW>();
        {   // conv3: 64 -> 64 -> global, in MFMA fragment order
            // (k = m*1024 + half*512 + lane*8 + j*4 + r, channel tile 2*half + j)
            f32x4 acc[MTW][NT3];
            conv_mma<VR, CL, 64, 18, NT3, 64>(lds, G::OFF2, gpos, nullptr, a.w3, w * NT3, lane, acc);
            u32x4 *dst = reinterpret_cast<u32x4 *>(a.act + b * (int64_t)(64 * G::P16)) + lane;
#pragma unroll
            for (int h = 0; h < NT3 / 2; h++) {
                const int half = w * (NT3 / 2) + h;
                const float b0 = bias3[2 * h], b1 = bias3[2 * h + 1];
#pragma unroll
                for (int m = 0; m < MTW; m++) {
                    u32x4 v;
                    v[0] = pack2(fmaxf(acc[m][2 * h][0] + b0, 0.0f), fmaxf(acc[m][2 * h][1] + b0, 0.0f));
                    v[1] = pack2(fmaxf(acc[m][2 * h][2] + b0, 0.0f), fmaxf(acc[m][2 * h][3] + b0, 0.0f));
                    v[2] = pack2(fmaxf(acc[m][2 * h + 1][0] + b1, 0.0f), fmaxf(acc[m][2 * h + 1][1] + b1, 0.0f));
                    v[3] = pack2(fmaxf(acc[m][2 * h + 1][2] + b1, 0.0f), fmaxf(acc[m][2 * h + 1][3] + b1, 0.0f));
                    dst[(m0 + m) * 128 + half * 64] = v;
                }
            }
        }
        if constexpr (!G::SEP) conv_sync<NW>();   // the next input image overwrites a2
    }
}

struct FcArgs {
    const uint16_t *act;     // [B][K] bf16, K = 64 * P16
    int64_t B;
    int K, A;
    const uint16_t *w4;      // fc1 [256][K] bf16
    const float *b4;
    const uint16_t *w5;      // fc2 [128][256] bf16
    const float *b5;
    const float *w6, *b6;    // fc3 [A][128], [A] fp32
    float *q, *feat;         // [B][A], [B][128] (feat may be null)
};

// ---- k_dqn_fc -----------------------------------------------------------
// 256 observations per workgroup, 8 waves x 32 rows. fc1 = [256 x K] x [K x 256]
// in k stages of 64: the stage's weight tile (256 x 64 bf16 = 32 KB) is staged
// through registers into one of two LDS buffers (loads issued a stage ahead,
// written after the stage's MFMAs, one barrier per stage), each B fragment read
// from LDS feeds two MFMAs (the wave's two row tiles); the A fragments (the
// conv3 activations) are loaded straight to registers a stage ahead. Tile image:
// [k32 plane][n][4 x 16 B], chunk c of row n stored at c ^ ((n >> 2) & 2): the
// 16 lanes of each ds_read_b128 lane group ({0-3,12-15,20-27}, ...) then hit
// distinct banks.
constexpr int kFcRowsPerWave = 32;
constexpr int kFcPlanes = 2;   // 32-wide k planes per stage (4: 128 KB of LDS, 89 VGPRs spilled)

__device__ __forceinline__ int fc_tile_off(int plane, int n, int c)
{
    return plane * 16384 + n * 64 + ((c ^ ((n >> 2) & 2)) << 4);
}

__global__ void __launch_bounds__(512) k_dqn_fc(const FcArgs a)
{
    constexpr int KP = kFcPlanes;
    __shared__ __attribute__((aligned(16))) uint8_t bt[2][KP * 16384];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int r16 = lane & 15, quad = lane >> 4, kq = 8 * quad;
    const int64_t row0 = (int64_t)blockIdx.x * kFcObs + wv * kFcRowsPerWave;
    // A rows of this lane (row tiles 0 and 1); rows past B read row 0 (results unused)
    // buffer descriptors: 32-bit lane offsets, the (row tile, stage, chunk) parts
    // as scalar offsets; the activation descriptor ends at the last valid row,
    // so rows past B read zeros
    const int64_t wg_row0 = (int64_t)blockIdx.x * kFcObs;
    const int64_t rows_here = a.B - wg_row0 < kFcObs ? a.B - wg_row0 : kFcObs;
    const auto rs_a = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(a.act + wg_row0 * a.K), 0,
                                                       (int)(rows_here * a.K * 2), 0x00020000);
    const auto rs_w = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(a.w4), 0, 256 * a.K * 2, 0x00020000);
    const int va = ((wv * kFcRowsPerWave + r16) * a.K + kq) * 2;
    // weight staging: slot = tid + 512 i -> row n = tid / (4 KP) + (128 / KP) i, 16-byte
    // chunk tid % (4 KP) of the stage
    constexpr int CPR = 4 * KP, RSTEP = 512 / CPR, NLB = 2 * KP;
    const int vw = ((tid / CPR) * a.K + (tid % CPR) * 8) * 2;
    const int wdst = fc_tile_off((tid % CPR) >> 2, tid / CPR, tid & 3);
    const int nstage = a.K / (32 * KP);
    u32x4 rb[NLB];
    bf16x8 a0[2][KP], a1[2][KP];   // A of even / odd stages (no register copies between stages)
    auto load_b = [&](int st) {
#pragma unroll
        for (int i = 0; i < NLB; i++)
            rb[i] = __builtin_amdgcn_raw_buffer_load_b128(rs_w, vw, i * RSTEP * a.K * 2 + st * 64 * KP, 0);
    };
    auto load_a = [&](int st, bf16x8 (&dst)[2][KP]) {
#pragma unroll
        for (int m = 0; m < 2; m++)
#pragma unroll
            for (int h = 0; h < KP; h++)
                dst[m][h] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                                           rs_a, va, m * 16 * a.K * 2 + st * 64 * KP + h * 64, 0));
    };
    auto store_b = [&](int buf) {
#pragma unroll
        for (int i = 0; i < NLB; i++) *reinterpret_cast<u32x4 *>(&bt[buf][wdst + RSTEP * 64 * i]) = rb[i];
    };
    f32x4 acc[2][16];
#pragma unroll
    for (int m = 0; m < 2; m++)
#pragma unroll
        for (int n = 0; n < 16; n++) acc[m][n] = (f32x4)0.0f;
    // stage st: MFMAs on A(st) (in ra) and the LDS tile st & 1; then the tile
    // st + 1 (loaded a stage ago) goes to LDS and A / B of stage st + 2 are issued
    auto stage = [&](int st, bf16x8 (&ra)[2][KP]) {
        const int buf = st & 1;
#pragma unroll
        for (int h = 0; h < KP; h++) {
#pragma unroll
            for (int n = 0; n < 16; n++) {
                const bf16x8 bv = *reinterpret_cast<const bf16x8 *>(&bt[buf][fc_tile_off(h, n * 16 + r16, quad)]);
                acc[0][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ra[0][h], bv, acc[0][n], 0, 0, 0);
                acc[1][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ra[1][h], bv, acc[1][n], 0, 0, 0);
            }
        }
        // unconditional (clamped) so the wait counts are the same on every path
        store_b(buf ^ 1);
        const int nx = st + 2 < nstage ? st + 2 : nstage - 1;
        load_b(nx);
        load_a(nx, ra);
        __syncthreads();
    };
    load_b(0);
    load_a(0, a0);
    store_b(0);
    load_b(nstage > 1 ? 1 : 0);
    load_a(nstage > 1 ? 1 : 0, a1);
    __syncthreads();
    int st = 0;
    for (; st + 1 < nstage; st += 2) {
        stage(st, a0);
        stage(st + 1, a1);
    }
    if (st < nstage) stage(st, a0);
    // fc2 and fc3: waves 0-3, then 4-7, each with a 16 KB slice of the tile buffers
    // (every wave passes one barrier: after its epilogue, or before it)
    if (wv >= 4) __syncthreads();
    {
        {
            uint8_t *hw = &bt[0][0] + (wv & 3) * 16384;
            // h1 = relu(fc1 + b) as bf16 [32][256] (16 KB): 16-byte chunk c of row r stored
            // at c ^ (r & 15), so the 16 rows of a fragment read hit distinct banks
#pragma unroll
            for (int n = 0; n < 16; n++) {
                const int col = n * 16 + r16;
                const float bb = a.b4[col];
#pragma unroll
                for (int m = 0; m < 2; m++)
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const int row = m * 16 + 4 * quad + r;
                        *reinterpret_cast<uint16_t *>(hw + row * 512 + (((col >> 3) ^ (row & 15)) << 4) + 2 * (col & 7)) =
                            (uint16_t)bf16_bits(fmaxf(acc[m][n][r] + bb, 0.0f));
                    }
            }
            wave_lds_sync();
            // fc2: [32 x 256] x [256 x 128]
            f32x4 acc2[2][8];
#pragma unroll
            for (int m = 0; m < 2; m++)
#pragma unroll
                for (int n = 0; n < 8; n++) acc2[m][n] = (f32x4)0.0f;
#pragma unroll
            for (int ks = 0; ks < 8; ks++) {
                bf16x8 av[2];
#pragma unroll
                for (int m = 0; m < 2; m++)
                    av[m] = *reinterpret_cast<const bf16x8 *>(hw + (m * 16 + r16) * 512 + (((ks * 4 + quad) ^ r16) << 4));
#pragma unroll
                for (int n = 0; n < 8; n++) {
                    const bf16x8 bv = *reinterpret_cast<const bf16x8 *>(a.w5 + (n * 16 + r16) * 256 + ks * 32 + kq);
                    acc2[0][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0], bv, acc2[0][n], 0, 0, 0);
                    acc2[1][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[1], bv, acc2[1][n], 0, 0, 0);
                }
            }
            wave_lds_sync();
            // h2 = relu(fc2 + b) fp32 [32][128] (16 KB), element k of row r at k ^ (r & 31)
            float *h2 = reinterpret_cast<float *>(hw);
#pragma unroll
            for (int n = 0; n < 8; n++) {
                const int col = n * 16 + r16;
                const float bb = a.b5[col];
#pragma unroll
                for (int m = 0; m < 2; m++)
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const int row = m * 16 + 4 * quad + r;
                        h2[row * 128 + (col ^ (row & 31))] = fmaxf(acc2[m][n][r] + bb, 0.0f);
                    }
            }
            wave_lds_sync();
            if (a.feat) {   // rows of 128 floats, two rows per pass (lanes 0-31, 32-63)
                for (int rr = 0; rr < kFcRowsPerWave; rr += 2) {
                    const int row = rr + (lane >> 5), c4 = (lane & 31) * 4;
                    if (row0 + row < a.B) {
                        f32x4 v;
#pragma unroll
                        for (int e = 0; e < 4; e++) v[e] = h2[row * 128 + ((c4 + e) ^ (row & 31))];
                        *reinterpret_cast<f32x4 *>(a.feat + (row0 + row) * 128 + c4) = v;
                    }
                }
            }
            for (int o = lane; o < kFcRowsPerWave * a.A; o += 64) {
                const int row = o / a.A, act = o - row * a.A;
                float sum = a.b6[act];
                const float *w6 = a.w6 + act * 128;
                for (int k = 0; k < 128; k++) sum = fmaf(h2[row * 128 + (k ^ (row & 31))], w6[k], sum);
                if (row0 + row < a.B) a.q[(row0 + row) * a.A + act] = sum;
            }
        }
    }
    if (wv < 4) __syncthreads();
}

}  // namespace dqn
}  // namespace snake

using namespace snake;
using namespace snake::dqn;

namespace {
typedef void (*conv_kernel_t)(ConvArgs);
struct ConvKernel {
    conv_kernel_t k;
    int nw;   // waves per observation (= workgroup size / 64)
};
template <int VR, int CL, int NW>
constexpr ConvKernel conv_kernel()
{
    if constexpr (NW == 4 && Geo<VR, CL>::MT % 2 != 0) return {k_dqn_conv<VR, CL, 2>, 2};   // odd tile count
    else return {k_dqn_conv<VR, CL, NW>, NW};
}
template <int NW>
struct ConvTable {
    ConvKernel k[5][3] = {
        {conv_kernel<1, 3, NW>(), conv_kernel<1, 4, NW>(), conv_kernel<1, 5, NW>()},
        {conv_kernel<2, 3, NW>(), conv_kernel<2, 4, NW>(), conv_kernel<2, 5, NW>()},
        {conv_kernel<3, 3, NW>(), conv_kernel<3, 4, NW>(), conv_kernel<3, 5, NW>()},
        {conv_kernel<4, 3, NW>(), conv_kernel<4, 4, NW>(), conv_kernel<4, 5, NW>()},
        {conv_kernel<5, 3, NW>(), conv_kernel<5, 4, NW>(), conv_kernel<5, 5, NW>()},
    };
};
const ConvTable<1> kConv1;
const ConvTable<2> kConv2;
const ConvTable<4> kConv4;
int g_conv_grid[3][5][3];
// waves per observation in k_dqn_conv when snake_dqn_cfg.conv_waves is 0: 4
// (two for odd row-tile counts). Forward at 262144 observations: 4.51 / 4.57 /
// 5.91 ms for 4 / 2 / 1 (conv_waves selects the others).
int conv_waves() { return 4; }
}  // namespace

extern "C" int snake_dqn_plan(const snake_dqn_cfg *cfg, snake_dqn_layout *out)
{
    if (!cfg || !out) { set_error("snake_dqn_plan: NULL argument"); return SNAKE_E_ARG; }
    const int H = cfg->height, W = cfg->width, C = cfg->channels, A = cfg->num_actions;
    if (H != W || H < 3 || H > 11 || !(H & 1)) {
        set_error("snake_dqn: the observation must be (2*vision_range+1)^2 with vision_range in [1, 5], got %dx%d", H, W);
        return SNAKE_E_CONFIG;
    }
    if (C < 8 || C > 32 || C % 8) {
        set_error("snake_dqn: channels must be 8 * frame_stack in [8, 32] (got %d)", C);
        return SNAKE_E_CONFIG;
    }
    if (A < 1 || A > 4) { set_error("snake_dqn: num_actions must be in [1, 4] (got %d)", A); return SNAKE_E_CONFIG; }
    if (cfg->conv_waves != 0 && cfg->conv_waves != 1 && cfg->conv_waves != 2 && cfg->conv_waves != 4) {
        set_error("snake_dqn: conv_waves must be 0, 1, 2 or 4 (got %d)", cfg->conv_waves);
        return SNAKE_E_CONFIG;
    }
    int cl = 3;
    while ((1 << cl) < C) cl++;
    const int MT = dqn_tiles(W), P16 = MT * 16, CP = 1 << cl;
    const int NB = (H + 2) * (W + 2);
    out->cpad = CP;
    out->p16 = P16;
    out->k1 = (9 * CP + 31) / 32 * 32;
    out->conv1_w = 32ll * out->k1;
    out->conv2_w = 64ll * 288;
    out->conv3_w = 64ll * 576;
    out->fc1_w = 256ll * 64 * P16;
    out->fc2_w = 128ll * 256;
    out->act_per_obs = 64ll * P16;
    const int CH = ((NB + 15) / 16) * 256;                       // Geo<>::CH, Geo<>::SEP
    const bool sep = 4 * ((12 + CP / 8) * CH + 2 * P16) <= 160 * 1024;
    out->lds_conv = (int32_t)((sep ? 12 + CP / 8 : 12) * CH + 2 * P16);
    return SNAKE_OK;
}

extern "C" int64_t snake_dqn_rows(const snake_dqn_cfg *cfg, int32_t *rows, int64_t n)
{
    snake_dqn_layout lay;
    const int rc = snake_dqn_plan(cfg, &lay);
    if (rc) return rc;
    if (rows) {
        if (n < lay.p16) { set_error("snake_dqn_rows: need %d entries", lay.p16); return SNAKE_E_ARG; }
        for (int i = 0; i < lay.p16; i++) rows[i] = -1;
        for (int p = 0; p < cfg->height * cfg->width; p++) rows[dqn_row_of(p, cfg->width)] = p;
    }
    return lay.p16;
}

extern "C" int snake_dqn_forward(const snake_dqn_cfg *cfg, const snake_dqn_net *net, const uint8_t *obs,
                                 int64_t batch, uint16_t *act_scratch, float *q_out, float *feat_out,
                                 void *stream)
{
    snake_dqn_layout lay;
    int rc = snake_dqn_plan(cfg, &lay);
    if (rc) return rc;
    if (!net || !obs || !act_scratch || !q_out || !net->conv1_w || !net->conv2_w || !net->conv3_w ||
        !net->fc1_w || !net->fc2_w || !net->conv1_b || !net->conv2_b || !net->conv3_b || !net->fc1_b ||
        !net->fc2_b || !net->fc3_w || !net->fc3_b) {
        set_error("snake_dqn_forward: NULL buffer");
        return SNAKE_E_ARG;
    }
    if (batch < 0) { set_error("snake_dqn_forward: batch < 0"); return SNAKE_E_ARG; }
    if (batch == 0) return SNAKE_OK;
    const hipStream_t s = (hipStream_t)stream;
    ConvArgs ca;
    ca.obs = obs; ca.B = batch; ca.C = cfg->channels;
    ca.w1 = net->conv1_w; ca.w2 = net->conv2_w; ca.w3 = net->conv3_w;
    ca.b1 = net->conv1_b; ca.b2 = net->conv2_b; ca.b3 = net->conv3_b;
    ca.act = act_scratch;
    const int vi = (cfg->height - 3) / 2, ci = lay.cpad == 8 ? 0 : (lay.cpad == 16 ? 1 : 2);
    const int want = cfg->conv_waves ? cfg->conv_waves : conv_waves();
    const ConvKernel ck = want == 1 ? kConv1.k[vi][ci] : (want == 4 ? kConv4.k[vi][ci] : kConv2.k[vi][ci]);
    const conv_kernel_t kc = ck.k;
    const int nw = ck.nw;
    int &grid = g_conv_grid[want == 1 ? 0 : (want == 2 ? 1 : 2)][vi][ci];
    if (!grid) {   // persistent grid: the resident workgroups of the whole device
        int per_cu = 0, dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)kc, 64 * nw, 0) != hipSuccess ||
            per_cu < 1 || cus < 1) {
            set_error("snake_dqn_forward: occupancy query failed");
            return SNAKE_E_LAUNCH;
        }
        grid = per_cu * cus;
    }
    const unsigned gconv = (unsigned)std::min<int64_t>(batch, grid);
    hipLaunchKernelGGL(kc, dim3(gconv), dim3(64 * nw), 0, s, ca);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) { set_error("k_dqn_conv launch failed: %s", hipGetErrorString(err)); return SNAKE_E_LAUNCH; }
    FcArgs fa;
    fa.act = act_scratch; fa.B = batch; fa.K = (int)lay.act_per_obs; fa.A = cfg->num_actions;
    fa.w4 = net->fc1_w; fa.b4 = net->fc1_b; fa.w5 = net->fc2_w; fa.b5 = net->fc2_b;
    fa.w6 = net->fc3_w; fa.b6 = net->fc3_b; fa.q = q_out; fa.feat = feat_out;
    const unsigned gfc = (unsigned)((batch + kFcObs - 1) / kFcObs);
    hipLaunchKernelGGL(k_dqn_fc, dim3(gfc), dim3(512), 0, s, fa);
    err = hipGetLastError();
    if (err != hipSuccess) { set_error("k_dqn_fc launch failed: %s", hipGetErrorString(err)); return SNAKE_E_LAUNCH; }
    return SNAKE_OK;
}
