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
// convolutions. The layer images live in LDS as NHWC bf16 with a zero border
// ((h+2) x (w+2) positions; a position's channels padded by 16 bytes so the 16
// lanes of one ds_read_b128 group hit distinct banks): the A fragment of tap
// (dy, dx) at output row p is one 16-byte read at a fixed offset from the row's
// own position, with no bounds checks, and with h, w and the channel counts
// compile-time that offset is an immediate. Each wave computes half the output
// channels (B fragments = weights from global memory, shared through L1/L2 by
// every workgroup) for all position tiles, so each A fragment feeds two MFMAs.
template <int VR, int CL>
struct Geo {
    static constexpr int W = 2 * VR + 1, H = W, P = H * W;
    static constexpr int MT = (P + 15) / 16, P16 = MT * 16;
    static constexpr int BW = W + 2, NB = BW * (H + 2);
    static constexpr int CP = 1 << CL;
    static constexpr int S0 = 2 * CP + (CP >= 16 ? 16 : 0);   // bytes per position: input image
    static constexpr int S1 = 2 * 32 + 16, S2 = 2 * 64 + 16;   // conv1 / conv2 output images
    static constexpr int K1S = (9 * CP + 31) / 32;              // conv1 k steps
    static constexpr int OFF1 = 0;                              // a1 [NB][S1]
    static constexpr int OFF2 = NB * S1;                        // a2 [NB][S2]; a0 [NB][S0] overlays it
    static constexpr int OFFT = OFF2 + NB * S2;                 // u16 [P16]: border index of row p
    static constexpr int LDS = OFFT + P16 * 2;
    static constexpr int NCELL0 = NB * CP / 8;                  // 16-byte cells of the input image
    static constexpr int NC = (NCELL0 + 127) / 128;             // per thread
    static constexpr int CENTER = (H / 2 + 1) * BW + W / 2 + 1;
    static constexpr int NBORDER = NB - P;
    __host__ __device__ static constexpr int bidx(int p) { return (p / W + 1) * BW + p % W + 1; }
    __host__ __device__ static constexpr int tapoff(int tap, int S) { return ((tap / 3) * BW + tap % 3) * S; }
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
// channel tiles starting at tile nt0. src / S: input border image and its
// position stride; tap offsets: per k step either compile-time (CIN >= 32: one
// tap per k step, the lane's 8 channels at 2 * kq bytes) or the lane's
// precomputed toff[ks], channel included (conv1 with CIN < 32).
template <int VR, int CL, int S, int CIN, int KS, int NTW>
__device__ __forceinline__ void conv_mma(const uint8_t *lds, int src, const int *gpos, const int *toff,
                                         const uint16_t *__restrict__ wt, int nt0, int lane,
                                         f32x4 (&acc)[Geo<VR, CL>::MT][NTW])
{
    using G = Geo<VR, CL>;
    const int r16 = lane & 15, kq = 8 * (lane >> 4);
    constexpr int K = KS * 32;
    int abase[G::MT];
#pragma unroll
    for (int m = 0; m < G::MT; m++) abase[m] = src + (gpos[m] - G::BW - 1) * S + (CIN >= 32 ? 2 * kq : 0);
#pragma unroll
    for (int m = 0; m < G::MT; m++)
#pragma unroll
        for (int j = 0; j < NTW; j++) acc[m][j] = (f32x4)0.0f;
    const uint16_t *wrow = wt + (nt0 * 16 + r16) * K + kq;
#pragma unroll
    for (int ks = 0; ks < KS; ks++) {
        bf16x8 bw[NTW];
#pragma unroll
        for (int j = 0; j < NTW; j++) bw[j] = *reinterpret_cast<const bf16x8 *>(wrow + j * 16 * K + ks * 32);
        int off;
        if constexpr (CIN >= 32) off = G::tapoff((ks * 32) / CIN, S) + 2 * ((ks * 32) % CIN);
        else off = toff[ks];
#pragma unroll
        for (int m = 0; m < G::MT; m++) {
            const bf16x8 av = *reinterpret_cast<const bf16x8 *>(lds + abase[m] + off);
#pragma unroll
            for (int j = 0; j < NTW; j++) acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bw[j], acc[m][j], 0, 0, 0);
        }
    }
}

// bias + ReLU -> bf16 into the interior of an NHWC border image (stride SD)
template <int VR, int CL, int SD, int NTW>
__device__ __forceinline__ void conv_store_lds(uint8_t *lds, int dst, const uint16_t *ptab, int nt0, int lane,
                                               const float *__restrict__ bias, f32x4 (&acc)[Geo<VR, CL>::MT][NTW])
{
    using G = Geo<VR, CL>;
    const int r16 = lane & 15, quad = lane >> 4;
#pragma unroll
    for (int j = 0; j < NTW; j++) {
        const int co = (nt0 + j) * 16 + r16;
        const float bb = bias[co];
#pragma unroll
        for (int m = 0; m < G::MT; m++) {
            const uint2 pq = *reinterpret_cast<const uint2 *>(ptab + m * 16 + 4 * quad);
            const uint32_t q[4] = {pq.x & 0xffffu, pq.x >> 16, pq.y & 0xffffu, pq.y >> 16};
#pragma unroll
            for (int r = 0; r < 4; r++) {
                if (m < G::MT - 1 || q[r] != 0xffffu)
                    *reinterpret_cast<uint16_t *>(lds + dst + q[r] * SD + 2 * co) =
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

template <int VR, int CL>
__global__ void __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(2))) k_dqn_conv(const ConvArgs a)
{
    using G = Geo<VR, CL>;
    __shared__ __attribute__((aligned(16))) uint8_t lds[G::LDS];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r16 = lane & 15, kq = 8 * (lane >> 4);
    uint16_t *ptab = reinterpret_cast<uint16_t *>(lds + G::OFFT);
    for (int p = tid; p < G::P16; p += 128) ptab[p] = p < G::P ? (uint16_t)G::bidx(p) : (uint16_t)0xffffu;
    for (int i = tid; i < G::NB * G::S1 / 16; i += 128) reinterpret_cast<u32x4 *>(lds + G::OFF1)[i] = (u32x4)0u;
    // gather rows (padding rows read the centre: finite values, results unused)
    int gpos[G::MT];
#pragma unroll
    for (int m = 0; m < G::MT; m++) {
        const int p = m * 16 + r16;
        gpos[m] = p < G::P ? G::bidx(p) : G::CENTER;
    }
    // conv1 per-lane tap offsets (k = tap * CP + channel; taps past the 9th meet zero weights)
    int toff1[G::K1S];
#pragma unroll
    for (int ks = 0; ks < G::K1S; ks++) {
        const int k0 = ks * 32 + kq, tap = k0 >> CL, ci = k0 & (G::CP - 1);
        toff1[ks] = tap < 9 ? G::tapoff(tap, G::S0) + 2 * ci : G::tapoff(4, G::S0);
    }
    // input cells of this thread: source byte offset within the observation, or -1 (zero)
    int csrc[G::NC], cdst[G::NC];
#pragma unroll
    for (int i = 0; i < G::NC; i++) {
        const int c = tid + 128 * i;
        const int q = c / (G::CP / 8), g = c % (G::CP / 8);
        const int y = q / G::BW - 1, x = q % G::BW - 1;
        const bool in = c < G::NCELL0 && (unsigned)y < (unsigned)G::H && (unsigned)x < (unsigned)G::W && g * 8 < a.C;
        csrc[i] = in ? (y * G::W + x) * a.C + g * 8 : -1;
        cdst[i] = c < G::NCELL0 ? G::OFF2 + q * G::S0 + g * 16 : -1;
    }
    uint2 xin[G::NC];
    auto load_obs = [&](int64_t b) {
        const uint8_t *x = a.obs + b * (int64_t)(G::P * a.C);
#pragma unroll
        for (int i = 0; i < G::NC; i++) xin[i] = csrc[i] >= 0 ? *reinterpret_cast<const uint2 *>(x + csrc[i]) : make_uint2(0, 0);
    };
    int64_t b = blockIdx.x;
    if (b < a.B) load_obs(b);
    __syncthreads();
    for (; b < a.B; b += gridDim.x) {
        // input image (whole, border included) over the a2 area
#pragma unroll
        for (int i = 0; i < G::NC; i++)
            if (cdst[i] >= 0) *reinterpret_cast<u32x4 *>(lds + cdst[i]) = bytes_to_bf16(xin[i]);
        if (b + gridDim.x < a.B) load_obs(b + gridDim.x);
        __syncthreads();
        {   // conv1: CP -> 32, wave w: channel tile w
            f32x4 acc[G::MT][1];
            conv_mma<VR, CL, G::S0, G::CP, G::K1S, 1>(lds, G::OFF2, gpos, toff1, a.w1, w, lane, acc);
            conv_store_lds<VR, CL, G::S1, 1>(lds, G::OFF1, ptab, w, lane, a.b1, acc);
        }
        __syncthreads();
        // the input image is dead: restore a2's zero border
        for (int i = tid; i < G::NBORDER * 8; i += 128) {
            const int bi = i >> 3, part = i & 7;
            int q;
            if (bi < G::BW) q = bi;
            else if (bi < 2 * G::BW) q = (G::H + 1) * G::BW + bi - G::BW;
            else q = (1 + ((bi - 2 * G::BW) >> 1)) * G::BW + ((bi - 2 * G::BW) & 1) * (G::BW - 1);
            *reinterpret_cast<u32x4 *>(lds + G::OFF2 + q * G::S2 + part * 16) = (u32x4)0u;
        }
        {   // conv2: 32 -> 64, wave w: channel tiles 2w, 2w+1
            f32x4 acc[G::MT][2];
            conv_mma<VR, CL, G::S1, 32, 9, 2>(lds, G::OFF1, gpos, nullptr, a.w2, 2 * w, lane, acc);
            conv_store_lds<VR, CL, G::S2, 2>(lds, G::OFF2, ptab, 2 * w, lane, a.b2, acc);
        }
        __syncthreads();
        {   // conv3: 64 -> 64 -> global, in MFMA fragment order (k = m*1024 + w*512 + lane*8 + j*4 + r)
            f32x4 acc[G::MT][2];
            conv_mma<VR, CL, G::S2, 64, 18, 2>(lds, G::OFF2, gpos, nullptr, a.w3, 2 * w, lane, acc);
            const float b0 = a.b3[(2 * w) * 16 + r16], b1 = a.b3[(2 * w + 1) * 16 + r16];
            u32x4 *dst = reinterpret_cast<u32x4 *>(a.act + b * (int64_t)(64 * G::P16)) + w * 64 + lane;
#pragma unroll
            for (int m = 0; m < G::MT; m++) {
                u32x4 v;
                v[0] = pack2(fmaxf(acc[m][0][0] + b0, 0.0f), fmaxf(acc[m][0][1] + b0, 0.0f));
                v[1] = pack2(fmaxf(acc[m][0][2] + b0, 0.0f), fmaxf(acc[m][0][3] + b0, 0.0f));
                v[2] = pack2(fmaxf(acc[m][1][0] + b1, 0.0f), fmaxf(acc[m][1][1] + b1, 0.0f));
                v[3] = pack2(fmaxf(acc[m][1][2] + b1, 0.0f), fmaxf(acc[m][1][3] + b1, 0.0f));
                dst[m * 128] = v;
            }
        }
        __syncthreads();
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
// [k32 plane][n][4 x 16 B], chunk c of row n stored at c ^ ((n >> 2) & 3) so
// the 16 rows of one ds_read_b128 lane group hit distinct banks.
constexpr int kFcRowsPerWave = 32;

__device__ __forceinline__ int fc_tile_off(int plane, int n, int c)
{
    return plane * 16384 + n * 64 + ((c ^ ((n >> 2) & 3)) << 4);
}

__global__ void __launch_bounds__(512) k_dqn_fc(const FcArgs a)
{
    __shared__ __attribute__((aligned(16))) uint8_t bt[2][32768];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int r16 = lane & 15, quad = lane >> 4, kq = 8 * quad;
    const int64_t row0 = (int64_t)blockIdx.x * kFcObs + wv * kFcRowsPerWave;
    // A rows of this lane (row tiles 0 and 1); rows past B read row 0 (results unused)
    const uint16_t *arow[2];
#pragma unroll
    for (int m = 0; m < 2; m++) {
        const int64_t r = row0 + m * 16 + r16;
        arow[m] = a.act + (r < a.B ? r : 0) * (int64_t)a.K + kq;
    }
    // weight staging: slot = tid + 512 i -> row n = slot / 8, 16-byte chunk c8 = slot % 8 of the stage
    const uint16_t *wsrc[4];
    int wdst[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int slot = tid + 512 * i, n = slot >> 3, c8 = slot & 7;
        wsrc[i] = a.w4 + (int64_t)n * a.K + c8 * 8;
        wdst[i] = fc_tile_off(c8 >> 2, n, c8 & 3);
    }
    const int nstage = a.K / 64;
    u32x4 rb[4];
    bf16x8 ra[2][2], an[2][2];
    auto load_b = [&](int st) {
#pragma unroll
        for (int i = 0; i < 4; i++) rb[i] = *reinterpret_cast<const u32x4 *>(wsrc[i] + st * 64);
    };
    auto load_a = [&](int st, bf16x8 (&dst)[2][2]) {
#pragma unroll
        for (int m = 0; m < 2; m++)
#pragma unroll
            for (int h = 0; h < 2; h++) dst[m][h] = *reinterpret_cast<const bf16x8 *>(arow[m] + st * 64 + h * 32);
    };
    auto store_b = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 4; i++) *reinterpret_cast<u32x4 *>(&bt[buf][wdst[i]]) = rb[i];
    };
    f32x4 acc[2][16];
#pragma unroll
    for (int m = 0; m < 2; m++)
#pragma unroll
        for (int n = 0; n < 16; n++) acc[m][n] = (f32x4)0.0f;
    load_b(0);
    load_a(0, ra);
    store_b(0);
    if (nstage > 1) { load_b(1); load_a(1, an); }
    __syncthreads();
    for (int st = 0; st < nstage; st++) {
        const int buf = st & 1;
#pragma unroll
        for (int h = 0; h < 2; h++) {
#pragma unroll
            for (int n = 0; n < 16; n++) {
                const bf16x8 bv = *reinterpret_cast<const bf16x8 *>(&bt[buf][fc_tile_off(h, n * 16 + r16, quad)]);
                acc[0][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ra[0][h], bv, acc[0][n], 0, 0, 0);
                acc[1][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ra[1][h], bv, acc[1][n], 0, 0, 0);
            }
        }
        if (st + 1 < nstage) {
            store_b(buf ^ 1);
#pragma unroll
            for (int m = 0; m < 2; m++)
#pragma unroll
                for (int h = 0; h < 2; h++) ra[m][h] = an[m][h];
            if (st + 2 < nstage) { load_b(st + 2); load_a(st + 2, an); }
        }
        __syncthreads();
    }
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
template <int VR, int CL>
constexpr conv_kernel_t conv_kernel() { return k_dqn_conv<VR, CL>; }
const conv_kernel_t kConvKernels[5][3] = {
    {conv_kernel<1, 3>(), conv_kernel<1, 4>(), conv_kernel<1, 5>()},
    {conv_kernel<2, 3>(), conv_kernel<2, 4>(), conv_kernel<2, 5>()},
    {conv_kernel<3, 3>(), conv_kernel<3, 4>(), conv_kernel<3, 5>()},
    {conv_kernel<4, 3>(), conv_kernel<4, 4>(), conv_kernel<4, 5>()},
    {conv_kernel<5, 3>(), conv_kernel<5, 4>(), conv_kernel<5, 5>()},
};
int g_conv_grid[5][3];
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
    int cl = 3;
    while ((1 << cl) < C) cl++;
    const int MT = (H * W + 15) / 16, P16 = MT * 16, CP = 1 << cl;
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
    out->lds_conv = (int32_t)(NB * (80 + 144) + 2 * P16);
    return SNAKE_OK;
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
    const conv_kernel_t kc = kConvKernels[vi][ci];
    if (!g_conv_grid[vi][ci]) {   // persistent grid: the resident workgroups of the whole device
        int per_cu = 0, dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)kc, 128, 0) != hipSuccess ||
            per_cu < 1 || cus < 1) {
            set_error("snake_dqn_forward: occupancy query failed");
            return SNAKE_E_LAUNCH;
        }
        g_conv_grid[vi][ci] = per_cu * cus;
    }
    const unsigned gconv = (unsigned)std::min<int64_t>(batch, g_conv_grid[vi][ci]);
    hipLaunchKernelGGL(kc, dim3(gconv), dim3(128), 0, s, ca);
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
