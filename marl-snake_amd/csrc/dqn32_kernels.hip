// dqn32_kernels.hip -- the fp32 mode of the fused consumer: the reference's DQN
// forward (train_dqn.py:104-151) in fp32 arithmetic on any observation size,
// including train_dqn.py's own 20x20 full-map Config (:29-33).
//
// Every layer is one GEMM launch
//
//   Y[m][n] = sum_k act(X)[m][k] * W[n][k]          (W row-major [N][K])
//
// on the fp32 matrix cores (v_mfma_f32_16x16x4_f32: exact fp32 products, fp32
// accumulation; gfx950's fp32 matrix and vector peaks are both 157 TF, the
// matrix form needs far fewer issue slots): k_conv32_mfma for the convolutions
// (A from an LDS patch of the input maps), k_fc32_mfma for fc1/fc2 (LDS-staged
// tiles). k_gemm32, a 128x64-tile GEMM on the vector ALUs, runs fc3 (A <= 64
// outputs) and the convolutions of maps too wide for the patch. The A operand is formed on
// the fly (no im2col buffer):
//   kConvU8   conv1: m = (b, y, x), k = (tap, ci); X = the uint8 NHWC
//             observation, zero outside the map (padding 1), / 255 when the
//             batch holds a value > 1 (train_dqn.py:122: x / 255 if x.max() > 1)
//   kConvF32  conv2/conv3: the previous layer's pre-activation NHWC, with its
//             bias and ReLU applied as it is read (zero padding after the ReLU)
//   kDense    fc1/fc2/fc3: relu(Y + bias[k % bmod]) of the previous layer; fc1's
//             weight columns are permuted once on the host from the reference's
//             NCHW flatten (ch*h*w + p) to NHWC (p*64 + ch)
// Layers store pre-activations; the last adds fc3's bias, forward_features is
// relu(fc2 + bias). Scratch: Y1 [B*P][32], Y2, Y3 [B*P][64], Y4 [B][256],
// Y5 [B][128] fp32 + a 16-byte flag word (snake_dqn32_scratch).
#include <hip/hip_runtime.h>

#include <stdint.h>

#include <stdlib.h>

#include <algorithm>

#include "snake_internal.h"

namespace snake {
namespace dqn32 {

enum { kConvU8 = 0, kConvF32 = 1, kDense = 2 };
constexpr int BM = 128, BN = 64, BK = 16, kThreads = 256;
struct GemmArgs {
    const void *x;          // A source (see mode)
    const float *xbias;     // bias applied (with ReLU) to the A source (modes 1, 2)
    int bmod;               // bias period along k (mode 2)
    const float *w;         // [N][K]
    float *y;               // [M][N]
    const float *ybias;     // added to the output (the last layer) or NULL
    int64_t M;
    int N, K;
    int H, W, C;            // conv geometry (modes 0, 1): map H x W, input channels C
    const int *scale_flag;  // mode 0: nonzero -> divide the uint8 input by 255
};

// One 128 x 64 output tile per 256-thread workgroup: thread (tx, ty) of 16 x 16
// owns rows ty*4 .. +3 and 64 + ty*4 .. +3 and columns tx*4 .. +3 (32 fp32
// accumulators; per k one 16-byte LDS read of each operand quad feeds 32 FMAs).
// The next k tile's global loads are issued before the current tile's FMAs.
template <int MODE>
__global__ void __launch_bounds__(kThreads) k_gemm32(const GemmArgs g)
{
    __shared__ __attribute__((aligned(16))) float As[BK][BM + 4];
    __shared__ __attribute__((aligned(16))) float Bs[BK][BN + 4];
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    const int64_t m0 = (int64_t)blockIdx.x * BM;
    const int n0 = blockIdx.y * BN;
    const int ar = tid >> 1, ak = (tid & 1) * 8;    // A loader: row ar, k ak .. ak+7
    const int br = tid >> 2, bk = (tid & 3) * 4;    // B loader: row br, k bk .. bk+3
    float acc[8][4] = {};
    float a[8], b[4];
    // A loader state: the row's map cell (conv modes) and the (tap, channel) of
    // its k offset, advanced by BK per tile without divisions
    const int64_t m = m0 + ar;
    const bool row_ok = m < g.M;
    int y = 0, x = 0, tap = 0, ci = 0;
    int64_t rowbase = 0;
    if constexpr (MODE != kDense) {
        const int P = g.H * g.W;
        const int64_t bb = row_ok ? m / P : 0;
        const int p = (int)(row_ok ? m - bb * P : 0);
        y = p / g.W;
        x = p - y * g.W;
        rowbase = ((bb * g.H + y) * g.W + x) * g.C;
        tap = ak / g.C;
        ci = ak - tap * g.C;
    } else {
        rowbase = m * g.K;
    }
    auto gather = [&](int k0, int c0, float (&v)[4]) {      // A[m][k0 .. k0+3], channel c0 (conv)
        v[0] = v[1] = v[2] = v[3] = 0.f;
        if (!row_ok || k0 >= g.K) return;
        if constexpr (MODE == kDense) {
            const float4 f = *reinterpret_cast<const float4 *>(reinterpret_cast<const float *>(g.x) + rowbase + k0);
            const float t[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const float u = t[i] + g.xbias[(k0 + i) & (g.bmod - 1)];
                v[i] = u > 0.f ? u : 0.f;
            }
        } else {
            const int dy = (tap * 11) >> 5, dx = tap - 3 * dy;      // tap / 3, tap % 3 for tap < 9
            const int yy = y + dy - 1, xx = x + dx - 1;
            if (yy < 0 || yy >= g.H || xx < 0 || xx >= g.W) return;   // zero padding
            const int64_t off = rowbase + (int64_t)(((dy - 1) * g.W + (dx - 1)) * g.C + c0);
            if constexpr (MODE == kConvU8) {
                const uchar4 u = *reinterpret_cast<const uchar4 *>(reinterpret_cast<const uint8_t *>(g.x) + off);
                v[0] = (float)u.x; v[1] = (float)u.y; v[2] = (float)u.z; v[3] = (float)u.w;
                if (*g.scale_flag) {
#pragma unroll
                    for (int i = 0; i < 4; i++) v[i] = v[i] / 255.0f;
                }
            } else {
                const float4 f = *reinterpret_cast<const float4 *>(reinterpret_cast<const float *>(g.x) + off);
                const float t[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const float u = t[i] + g.xbias[c0 + i];
                    v[i] = u > 0.f ? u : 0.f;
                }
            }
        }
    };
    auto load = [&](int k0) {
        float t0[4], t1[4];
        gather(k0 + ak, ci, t0);
        gather(k0 + ak + 4, ci + 4, t1);          // same tap: C % 8 == 0
        if constexpr (MODE != kDense) {
            ci += BK;
            while (ci >= g.C) { ci -= g.C; tap++; }
        }
#pragma unroll
        for (int i = 0; i < 4; i++) { a[i] = t0[i]; a[4 + i] = t1[i]; }
        const int n = n0 + br, kk = k0 + bk;
        b[0] = b[1] = b[2] = b[3] = 0.f;
        if (n < g.N && kk < g.K) {
            const float *wr = g.w + (int64_t)n * g.K + kk;
            if (kk + 4 <= g.K) {
                const float4 f = *reinterpret_cast<const float4 *>(wr);
                b[0] = f.x; b[1] = f.y; b[2] = f.z; b[3] = f.w;
            } else {
#pragma unroll
                for (int i = 0; i < 4; i++) b[i] = (kk + i < g.K) ? wr[i] : 0.f;
            }
        }
    };
    auto store = [&]() {
#pragma unroll
        for (int i = 0; i < 8; i++) As[ak + i][ar] = a[i];
#pragma unroll
        for (int i = 0; i < 4; i++) Bs[bk + i][br] = b[i];
    };
    load(0);
    store();
    __syncthreads();
    for (int k0 = 0; k0 < g.K; k0 += BK) {
        const bool more = k0 + BK < g.K;
        if (more) load(k0 + BK);
#pragma unroll
        for (int k = 0; k < BK; k++) {
            const float4 a0 = *reinterpret_cast<const float4 *>(&As[k][ty * 4]);
            const float4 a1 = *reinterpret_cast<const float4 *>(&As[k][64 + ty * 4]);
            const float4 bq = *reinterpret_cast<const float4 *>(&Bs[k][tx * 4]);
            const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
            const float bv[4] = {bq.x, bq.y, bq.z, bq.w};
#pragma unroll
            for (int i = 0; i < 8; i++)
#pragma unroll
                for (int j = 0; j < 4; j++) acc[i][j] = __builtin_fmaf(av[i], bv[j], acc[i][j]);
        }
        __syncthreads();
        if (more) {
            store();
            __syncthreads();
        }
    }
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const int64_t m = m0 + (i < 4 ? ty * 4 + i : 64 + ty * 4 + i - 4);
        if (m >= g.M) continue;
        const int n = n0 + tx * 4;
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; j++) o[j] = acc[i][j] + ((g.ybias && n + j < g.N) ? g.ybias[n + j] : 0.f);
        if (n + 4 <= g.N && (g.N & 3) == 0) {
            *reinterpret_cast<float4 *>(g.y + m * g.N + n) = make_float4(o[0], o[1], o[2], o[3]);
        } else {
#pragma unroll
            for (int j = 0; j < 4; j++)
                if (n + j < g.N) g.y[m * g.N + n + j] = o[j];
        }
    }
}

// ------------------------------------------------------------------------
// The convolutions on the fp32 matrix cores (v_mfma_f32_16x16x4_f32: exact fp32
// products, fp32 accumulation). Implicit GEMM, rows = output positions of the
// batch flattened (b, y, x), columns = output channels, k = (tap, ci).
//
// The A operand comes from an LDS patch, not from global gathers: the batch's
// maps are seen as one tall image, map b's row y at tall row b*(H+1)+y+1, with
// one zero row between maps (and above the first), so a 3x3 tap never needs a
// bounds test. A workgroup's 128 consecutive rows need tall rows
// [T(m0)-1, T(m0+127)+1] x all W+2 bordered columns; they are staged once,
// with the previous layer's bias and ReLU (or the uint8 scaling) applied and
// zeros written for borders, separators and rows past the batch. A cell holds
// C channels padded to conv_cell_stride(C) floats (bank-conflict-free
// ds_read_b128 rows).
//
// MFMA k order: in a 16-k block, lane group g = lane/16 owns k0+4g .. k0+4g+3
// and MFMA j of the block takes k0+4g+j from every group, so one ds_read_b128
// (A: four consecutive channels of one cell) and one 16-byte global load (B: W
// row-major [N][K]) feed four MFMAs. Output fragment: lane l, register r ->
// row 4*(l/16)+r, column l%16.
constexpr int kConvRows = 128;
constexpr int kPatchMaxBytes = 80 * 1024;   // two workgroups per CU

__host__ __device__ inline int conv_patch_rows(int H, int W)
{
    // tall rows spanned by 128 consecutive positions + the two halo rows
    const int P = H * W;
    return (kConvRows - 1 + W - 1) / W + 1 + (kConvRows - 1 + P - 1) / P + 2;
}

// Cell stride in floats: C + 8 when C % 16 == 0, else C (C % 8 == 0), so that the
// stride in 16-byte slots is 2 mod 4. ds_read_b128 serves a wave in four lane
// groups of 16 ({0-3,12-15,20-27}, {4-11,16-19,28-31}, and the upper half
// alike: MI355X_MICROARCH.md §LDS); a group holds 8 rows of lane group g and
// 8 of g+1, distinct mod 8, so their slots 2m*row + g are all distinct (a
// stride of 1 mod 4 made every group 2-way).
__host__ __device__ inline int conv_cell_stride(int C) { return C + ((C & 15) ? 0 : 8); }

__host__ inline int64_t conv_patch_bytes(int H, int W, int C)
{
    return (int64_t)conv_patch_rows(H, W) * (W + 2) * conv_cell_stride(C) * 4;
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

// NT = output channels / 16 (2: conv1, 4: conv2/conv3). Wave w takes column
// tile w % NT and 16*NT/... row tiles: NT == 4 -> all 8 row tiles, NT == 2 ->
// row tiles 4*(w/2) .. +3. WT (NT == 4 only): wave tiles of 4 row x 2 column
// tiles instead -- wave w takes column tiles 2*(w%2), +1 and row tiles
// 4*(w/2) .. +3: each A fragment feeds two MFMAs (half the LDS reads per MFMA),
// each block loads two B fragments.
template <int MODE, int NT, bool WT = false>
__global__ void __launch_bounds__(256) k_conv32_mfma(const GemmArgs g)
{
    static_assert(!WT || NT == 4, "wave tiles of 4 x 2 need four column tiles");
    extern __shared__ __attribute__((aligned(16))) float patch[];
    __shared__ int offs[4 * 76];   // K <= 9 * 128: 72 blocks + padding + 1
    constexpr int RT = WT ? 4 : (NT == 4 ? 8 : 4);   // row tiles per wave
    constexpr int CT = WT ? 2 : 1;                   // column tiles per wave
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int H = g.H, W = g.W, C = g.C, K = g.K, N = g.N;
    const int W2 = W + 2, CS = conv_cell_stride(C), P = H * W;
    const int64_t M = g.M, m0 = (int64_t)blockIdx.x * kConvRows;
    const int64_t B = M / P;
    // tall row of the first position
    const int64_t b0 = m0 / P;
    const int p0 = (int)(m0 - b0 * P);
    const int64_t t0 = b0 * (H + 1) + p0 / W + 1 - 1;   // first patch row (halo above)
    const int PR = conv_patch_rows(H, W);
    // ---- stage the patch: cell (r, c) = tall row t0 + r, bordered column c
    const int C4 = C >> 2, cells = PR * W2;
    float scale = 1.f;
    if constexpr (MODE == kConvU8) scale = *g.scale_flag ? (1.f / 255.f) : 1.f;
    // 8 loads in flight per thread, then the conversions and LDS stores
    constexpr int kBatch = 8;
    const int total = cells * C4;
    for (int q0 = tid; q0 < total; q0 += 256 * kBatch) {
        f32x4 v[kBatch];
        int dst[kBatch];
        bool live[kBatch];
#pragma unroll
        for (int u = 0; u < kBatch; u++) {
            const int q = q0 + 256 * u;
            const int cell = q / C4, c4 = q - cell * C4;
            const int r = cell / W2, c = cell - r * W2;
            const int64_t t = t0 + r;
            const int64_t b = t / (H + 1);
            const int yy = (int)(t - b * (H + 1)) - 1, xx = c - 1;
            dst[u] = q < total ? cell * CS + 4 * c4 : -1;
            // unconditional loads (element 0 for cells outside the maps, zeroed
            // below): a load under a branch is waited for inside the branch
            live[u] = q < total && yy >= 0 && xx >= 0 && xx < W && b < B;
            const int64_t off = live[u] ? ((b * H + yy) * W + xx) * C + 4 * c4 : 0;
            if constexpr (MODE == kConvU8) {
                const uchar4 uc = *reinterpret_cast<const uchar4 *>(reinterpret_cast<const uint8_t *>(g.x) + off);
                v[u].x = (float)uc.x; v[u].y = (float)uc.y; v[u].z = (float)uc.z; v[u].w = (float)uc.w;
            } else {
                v[u] = *reinterpret_cast<const f32x4 *>(reinterpret_cast<const float *>(g.x) + off);
            }
        }
#pragma unroll
        for (int u = 0; u < kBatch; u++) {
            f32x4 w = v[u];
            if constexpr (MODE == kConvU8) {
                // (the reference divides: x / 255)
                if (scale != 1.f) { w.x = w.x / 255.0f; w.y = w.y / 255.0f; w.z = w.z / 255.0f; w.w = w.w / 255.0f; }
            } else {
                const int c4 = (q0 + 256 * u) % C4;
                const float *bb = g.xbias + 4 * c4;   // (the caller's bias: no alignment assumed)
                w.x += bb[0]; w.y += bb[1]; w.z += bb[2]; w.w += bb[3];
                w.x = w.x > 0.f ? w.x : 0.f; w.y = w.y > 0.f ? w.y : 0.f;
                w.z = w.z > 0.f ? w.z : 0.f; w.w = w.w > 0.f ? w.w : 0.f;
            }
            if (!live[u]) w = (f32x4){0.f, 0.f, 0.f, 0.f};
            if (dst[u] >= 0) *reinterpret_cast<f32x4 *>(patch + dst[u]) = w;
        }
    }
    __syncthreads();
    // ---- this wave's tiles
    const int ct = WT ? 2 * (wave & 1) : wave % NT;
    const int rt0 = WT ? 4 * (wave >> 1) : (NT == 4 ? 0 : 4 * (wave / 2));
    const int grp = lane >> 4, l16 = lane & 15;
    int abase[RT];   // LDS 16-byte index of each row tile's lane-row cell (tap (1,1), channel 0)
#pragma unroll
    for (int i = 0; i < RT; i++) {
        int64_t m = m0 + (rt0 + i) * 16 + l16;
        if (m >= M) m = M - 1;   // computed, never stored
        const int64_t b = m / P;
        const int p = (int)(m - b * P), y = p / W, x = p - y * W;
        const int r = (int)(b * (H + 1) + y + 1 - t0);
        abase[i] = ((r * W2 + x + 1) * CS) >> 2;
    }
    int col[CT];
    const float *wrow[CT];
#pragma unroll
    for (int c = 0; c < CT; c++) {
        col[c] = (ct + c) * 16 + l16;
        wrow[c] = g.w + (int64_t)col[c] * K;
    }
    f32x4 acc[RT][CT];
#pragma unroll
    for (int i = 0; i < RT; i++)
#pragma unroll
        for (int c = 0; c < CT; c++) acc[i][c] = (f32x4){0.f, 0.f, 0.f, 0.f};
    // per 16-k block and lane group: the LDS offset (in 16-byte units) of its
    // (tap, channel) from a row's centre cell; blocks are processed kRing at a
    // time, and k past K (the padding blocks, one extra entry for the last
    // prefetch) reads the centre cell with a zero B operand
    constexpr int kRing = 2;
    const int nb = (K + 15) >> 4, nbp = (nb + kRing - 1) / kRing * kRing;
    for (int q = tid; q < 4 * (nbp + 1); q += 256) {
        const int kq = 4 * q;
        int o = 0;
        if (kq < K) {
            const int tap = kq / C, ci = kq - tap * C;
            const int dy = (tap * 11) >> 5, dx = tap - 3 * dy;
            o = (((dy - 1) * W2 + (dx - 1)) * CS + ci) >> 2;
        }
        offs[q] = o;
    }
    __syncthreads();
    // B: kRing blocks of loads in flight (unconditional, clamped addresses);
    // A: the next block's fragments are read before this block's MFMAs
    const f32x4 *patch4 = reinterpret_cast<const f32x4 *>(patch);
    const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
    f32x4 bq[kRing][CT];
#pragma unroll
    for (int d = 0; d < kRing; d++)
#pragma unroll
        for (int c = 0; c < CT; c++)
            bq[d][c] = *reinterpret_cast<const f32x4 *>(wrow[c] + min(16 * d + 4 * grp, K - 4));
    f32x4 a[RT];
    {
        const int off = offs[grp];
#pragma unroll
        for (int i = 0; i < RT; i++) a[i] = patch4[abase[i] + off];
    }
    // two blocks per iteration: the B ring and the A fragments ping-pong
    // between fixed registers (a register copy would wait for the load it copies)
    f32x4 a2[RT];
    auto block = [&](int kb, f32x4 (&acur)[RT], f32x4 (&anext)[RT], f32x4 (&bslot)[CT]) {
        const int off = offs[4 * (kb + 1) + grp];
#pragma unroll
        for (int i = 0; i < RT; i++) anext[i] = patch4[abase[i] + off];
        // (conv2/conv3: K = 9 * 32 or 9 * 64, a multiple of 16 -- no mask, so
        // nothing ties the ring's loads to a select at issue time)
        f32x4 bv[CT];
#pragma unroll
        for (int c = 0; c < CT; c++) {
            bv[c] = bslot[c];
            if constexpr (MODE == kConvU8) bv[c] = 16 * kb + 4 * grp < K ? bv[c] : zero;
            bslot[c] = *reinterpret_cast<const f32x4 *>(wrow[c] + min(16 * (kb + kRing) + 4 * grp, K - 4));
        }
        // (the loads stay issued ahead of this block's MFMAs: without the
        // barriers the scheduler sinks them next to their uses)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < 4; j++)
#pragma unroll
            for (int i = 0; i < RT; i++)
#pragma unroll
                for (int c = 0; c < CT; c++)
                    acc[i][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(acur[i][j], bv[c][j], acc[i][c], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    };
    for (int kb = 0; kb < nbp; kb += 2) {
        block(kb, a, a2, bq[0]);
        block(kb + 1, a2, a, bq[1]);
    }
    // ---- pre-activations out: Y[m][n]
#pragma unroll
    for (int i = 0; i < RT; i++) {
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int64_t m = m0 + (rt0 + i) * 16 + 4 * grp + r;
#pragma unroll
            for (int c = 0; c < CT; c++)
                if (m < M) g.y[m * N + col[c]] = acc[i][c][r];
        }
    }
}

template <int MODE, int NT>
int conv_mfma(const GemmArgs &g, hipStream_t s, const char *what)
{
    const int64_t lds = conv_patch_bytes(g.H, g.W, g.C);
    const dim3 grid((unsigned)((g.M + kConvRows - 1) / kConvRows));
    // 4 x 2 wave tiles for the 64-channel layers (20x20x8, 16 384 observations:
    // conv2/conv3 3 715 -> 3 666 us per launch on average against 8 x 1, forward
    // 9.84 -> 9.75 ms; parity green)
    if constexpr (NT == 4) hipLaunchKernelGGL((k_conv32_mfma<MODE, 4, true>), grid, dim3(256), (size_t)lds, s, g);
    else hipLaunchKernelGGL((k_conv32_mfma<MODE, NT>), grid, dim3(256), (size_t)lds, s, g);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) { set_error("%s launch failed: %s", what, hipGetErrorString(err)); return SNAKE_E_LAUNCH; }
    return SNAKE_OK;
}

// The dense layers with N a multiple of 128 (fc1: 64hw -> 256, fc2: 256 -> 128)
// on the fp32 matrix cores: Y = relu(X + bias[k % bmod]) W^T. A workgroup of
// 8 waves owns 128 rows x 128 columns; wave (rg, cg) = (w % 4, w / 4) owns rows
// 32 rg .. +31 and columns 64 cg .. +63 (2 x 4 tiles of 16 x 16). Per 32-k block
// the A tile (bias and ReLU applied once) and the W tile are staged in LDS,
// double-buffered: the next block's global loads are issued before this
// block's MFMAs and stored after them, one barrier per block. Rows of 32 k
// padded to 40 floats: the row lanes of a ds_read_b128 group hit distinct banks.
constexpr int kFcK = 32, kFcS = kFcK + 8;   // rows of 10 slots: 2 mod 4 (see conv_cell_stride)

__global__ void __launch_bounds__(512) k_fc32_mfma(const GemmArgs g)
{
    __shared__ __attribute__((aligned(16))) float As[2][128 * kFcS];
    __shared__ __attribute__((aligned(16))) float Bs[2][128 * kFcS];
    __shared__ __attribute__((aligned(16))) float bias[256];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int rg = wave & 3, cg = wave >> 2, grp = lane >> 4, l16 = lane & 15;
    const int K = g.K, N = g.N;
    const int64_t M = g.M;
    for (int q = tid; q < g.bmod; q += 512) bias[q] = g.xbias[q];
    const int64_t m0 = (int64_t)blockIdx.x * 128;
    const int n0 = blockIdx.y * 128;
    // stager: thread t loads float4 (row t/8 and 64 + t/8, k 4*(t%8)) of A and of W
    const int sr = tid >> 3, sk = 4 * (tid & 7);
    const float *ap[2];
    const float *wp[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
        int64_t m = m0 + sr + 64 * h;
        if (m >= M) m = M - 1;   // computed, never stored
        ap[h] = reinterpret_cast<const float *>(g.x) + m * K + sk;
        wp[h] = g.w + (int64_t)(n0 + sr + 64 * h) * K + sk;
    }
    const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
    f32x4 ra[2], rw[2];
    auto fetch = [&](int k0) {
        const bool ok = k0 + sk < K;
#pragma unroll
        for (int h = 0; h < 2; h++) {
            ra[h] = ok ? *reinterpret_cast<const f32x4 *>(ap[h] + k0) : zero;
            rw[h] = ok ? *reinterpret_cast<const f32x4 *>(wp[h] + k0) : zero;
        }
    };
    const int bm = g.bmod - 1;
    auto stage = [&](int buf, int k0) {
        const f32x4 bv = *reinterpret_cast<const f32x4 *>(&bias[(k0 + sk) & bm]);
#pragma unroll
        for (int h = 0; h < 2; h++) {
            f32x4 a;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const float u = ra[h][j] + bv[j];
                a[j] = u > 0.f ? u : 0.f;   // (k past K: W is zero there)
            }
            *reinterpret_cast<f32x4 *>(&As[buf][(sr + 64 * h) * kFcS + sk]) = a;
            *reinterpret_cast<f32x4 *>(&Bs[buf][(sr + 64 * h) * kFcS + sk]) = rw[h];
        }
    };
    f32x4 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int c = 0; c < 4; c++) acc[i][c] = zero;
    fetch(0);
    __syncthreads();   // bias
    stage(0, 0);
    __syncthreads();
    const int nb = (K + kFcK - 1) / kFcK;
    for (int kb = 0; kb < nb; kb++) {
        const int cur = kb & 1;
        if (kb + 1 < nb) fetch((kb + 1) * kFcK);
#pragma unroll
        for (int h = 0; h < 2; h++) {
            f32x4 a[2], b[4];
#pragma unroll
            for (int i = 0; i < 2; i++)
                a[i] = *reinterpret_cast<const f32x4 *>(&As[cur][(rg * 32 + i * 16 + l16) * kFcS + 16 * h + 4 * grp]);
#pragma unroll
            for (int c = 0; c < 4; c++)
                b[c] = *reinterpret_cast<const f32x4 *>(&Bs[cur][(cg * 64 + c * 16 + l16) * kFcS + 16 * h + 4 * grp]);
#pragma unroll
            for (int j = 0; j < 4; j++)
#pragma unroll
                for (int i = 0; i < 2; i++)
#pragma unroll
                    for (int c = 0; c < 4; c++)
                        acc[i][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][j], b[c][j], acc[i][c], 0, 0, 0);
        }
        if (kb + 1 < nb) stage(cur ^ 1, (kb + 1) * kFcK);
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const int n = n0 + cg * 64 + c * 16 + l16;
            const float yb = g.ybias ? g.ybias[n] : 0.f;
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int64_t m = m0 + rg * 32 + i * 16 + 4 * grp + r;
                if (m < M) g.y[m * N + n] = acc[i][c][r] + yb;
            }
        }
}

int fc_mfma(const GemmArgs &g, hipStream_t s, const char *what)
{
    const dim3 grid((unsigned)((g.M + 127) / 128), (unsigned)(g.N / 128));
    hipLaunchKernelGGL(k_fc32_mfma, grid, dim3(512), 0, s, g);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) { set_error("%s launch failed: %s", what, hipGetErrorString(err)); return SNAKE_E_LAUNCH; }
    return SNAKE_OK;
}

// flag = any observation byte > 1 (the reference's x.max() > 1.0 test)
__global__ void k_obs_max(const uint8_t *obs, int64_t n, int *flag)
{
    int hit = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        hit |= obs[i] > 1;
    if (__any(hit) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

// forward_features = relu(fc2 pre-activation + bias)
__global__ void k_bias_relu(const float *y, const float *bias, int n, int64_t total, float *out)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < total) {
        const float t = y[i] + bias[i % n];
        out[i] = t > 0.f ? t : 0.f;
    }
}

template <int MODE>
int gemm(const GemmArgs &g, hipStream_t s, const char *what)
{
    const dim3 grid((unsigned)((g.M + BM - 1) / BM), (unsigned)((g.N + BN - 1) / BN));
    hipLaunchKernelGGL(k_gemm32<MODE>, grid, dim3(kThreads), 0, s, g);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) { set_error("%s launch failed: %s", what, hipGetErrorString(err)); return SNAKE_E_LAUNCH; }
    return SNAKE_OK;
}

int check_cfg(const snake_dqn_cfg *cfg)
{
    if (!cfg) { set_error("snake_dqn32: NULL cfg"); return SNAKE_E_ARG; }
    if (cfg->height < 1 || cfg->width < 1 || cfg->height > 255 || cfg->width > 255) {
        set_error("snake_dqn32: observation %dx%d out of range", cfg->height, cfg->width);
        return SNAKE_E_CONFIG;
    }
    if (cfg->channels < 8 || cfg->channels % 8 || cfg->channels > 128) {
        set_error("snake_dqn32: channels must be a multiple of 8 in [8, 128] (got %d)", cfg->channels);
        return SNAKE_E_CONFIG;
    }
    if (cfg->num_actions < 1 || cfg->num_actions > 64) {
        set_error("snake_dqn32: num_actions must be in [1, 64] (got %d)", cfg->num_actions);
        return SNAKE_E_CONFIG;
    }
    return SNAKE_OK;
}

// scratch layout (bytes): flag (16) | Y1 | Y2 | Y3 | Y4 | Y5
struct Scratch {
    int *flag;
    float *y1, *y2, *y3, *y4, *y5;
};

int64_t scratch_bytes(const snake_dqn_cfg *cfg, int64_t B, void *base, Scratch *out)
{
    const int64_t P = (int64_t)cfg->height * cfg->width;
    const int64_t n1 = B * P * 32, n2 = B * P * 64, n3 = n2, n4 = B * 256, n5 = B * 128;
    if (out) {
        uint8_t *p = reinterpret_cast<uint8_t *>(base);
        out->flag = reinterpret_cast<int *>(p);
        out->y1 = reinterpret_cast<float *>(p + 16);
        out->y2 = out->y1 + n1;
        out->y3 = out->y2 + n2;
        out->y4 = out->y3 + n3;
        out->y5 = out->y4 + n4;
    }
    return 16 + 4 * (n1 + n2 + n3 + n4 + n5);
}

}  // namespace dqn32
}  // namespace snake

using namespace snake;

extern "C" int64_t snake_dqn32_scratch(const snake_dqn_cfg *cfg, int64_t batch)
{
    const int rc = dqn32::check_cfg(cfg);
    if (rc) return rc;
    if (batch < 0) { set_error("snake_dqn32_scratch: batch < 0"); return SNAKE_E_ARG; }
    return dqn32::scratch_bytes(cfg, batch, nullptr, nullptr);
}

extern "C" int snake_dqn32_forward(const snake_dqn_cfg *cfg, const snake_dqn32_net *net, const uint8_t *obs,
                                   int64_t batch, void *scratch, float *q_out, float *feat_out, void *stream)
{
    int rc = dqn32::check_cfg(cfg);
    if (rc) return rc;
    if (!net || !obs || !scratch || !q_out || !net->conv1_w || !net->conv2_w || !net->conv3_w || !net->fc1_w ||
        !net->fc2_w || !net->fc3_w || !net->conv1_b || !net->conv2_b || !net->conv3_b || !net->fc1_b ||
        !net->fc2_b || !net->fc3_b) {
        set_error("snake_dqn32_forward: NULL buffer");
        return SNAKE_E_ARG;
    }
    if (batch < 0) { set_error("snake_dqn32_forward: batch < 0"); return SNAKE_E_ARG; }
    if (batch == 0) return SNAKE_OK;
    const hipStream_t s = (hipStream_t)stream;
    dqn32::Scratch sc;
    dqn32::scratch_bytes(cfg, batch, scratch, &sc);
    const int H = cfg->height, W = cfg->width, C = cfg->channels, A = cfg->num_actions;
    const int64_t P = (int64_t)H * W, BP = batch * P;
    if (hipMemsetAsync(sc.flag, 0, 16, s) != hipSuccess) { set_error("snake_dqn32: memset failed"); return SNAKE_E_LAUNCH; }
    {
        const int64_t n = BP * C;
        const unsigned blocks = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
        hipLaunchKernelGGL(dqn32::k_obs_max, dim3(blocks), dim3(256), 0, s, obs, n, sc.flag);
        if (hipGetLastError() != hipSuccess) { set_error("k_obs_max launch failed"); return SNAKE_E_LAUNCH; }
    }
    dqn32::GemmArgs g{};
    g.H = H; g.W = W;
    // the convolutions on the matrix cores when the widest layer's LDS patch
    // fits (every map up to ~40 wide), else the vector-ALU GEMM
    const bool mfma = dqn32::conv_patch_bytes(H, W, std::max(C, 64)) <= dqn32::kPatchMaxBytes;
    // conv1: uint8 NHWC obs -> Y1 [B*P][32]
    g.x = obs; g.xbias = nullptr; g.w = net->conv1_w; g.y = sc.y1; g.ybias = nullptr;
    g.M = BP; g.N = 32; g.K = 9 * C; g.C = C; g.scale_flag = sc.flag;
    if ((rc = mfma ? dqn32::conv_mfma<dqn32::kConvU8, 2>(g, s, "conv1") : dqn32::gemm<dqn32::kConvU8>(g, s, "conv1")))
        return rc;
    // conv2: relu(Y1 + b1) -> Y2 [B*P][64]
    g.x = sc.y1; g.xbias = net->conv1_b; g.w = net->conv2_w; g.y = sc.y2;
    g.N = 64; g.K = 9 * 32; g.C = 32;
    if ((rc = mfma ? dqn32::conv_mfma<dqn32::kConvF32, 4>(g, s, "conv2") : dqn32::gemm<dqn32::kConvF32>(g, s, "conv2")))
        return rc;
    // conv3: relu(Y2 + b2) -> Y3
    g.x = sc.y2; g.xbias = net->conv2_b; g.w = net->conv3_w; g.y = sc.y3;
    g.N = 64; g.K = 9 * 64; g.C = 64;
    if ((rc = mfma ? dqn32::conv_mfma<dqn32::kConvF32, 4>(g, s, "conv3") : dqn32::gemm<dqn32::kConvF32>(g, s, "conv3")))
        return rc;
    // fc1: relu(Y3 + b3) flattened NHWC (P*64) -> Y4 [B][256]
    g.x = sc.y3; g.xbias = net->conv3_b; g.bmod = 64; g.w = net->fc1_w; g.y = sc.y4;
    g.M = batch; g.N = 256; g.K = (int)(P * 64);
    if ((rc = dqn32::fc_mfma(g, s, "fc1"))) return rc;
    // fc2: relu(Y4 + bfc1) -> Y5 [B][128]
    g.x = sc.y4; g.xbias = net->fc1_b; g.bmod = 256; g.w = net->fc2_w; g.y = sc.y5;
    g.N = 128; g.K = 256;
    if ((rc = dqn32::fc_mfma(g, s, "fc2"))) return rc;
    // fc3: relu(Y5 + bfc2) -> q [B][A] + bfc3
    g.x = sc.y5; g.xbias = net->fc2_b; g.bmod = 128; g.w = net->fc3_w; g.y = q_out; g.ybias = net->fc3_b;
    g.N = A; g.K = 128;
    if ((rc = dqn32::gemm<dqn32::kDense>(g, s, "fc3"))) return rc;
    if (feat_out) {
        const int64_t total = batch * 128;
        hipLaunchKernelGGL(dqn32::k_bias_relu, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, sc.y5,
                           net->fc2_b, 128, total, feat_out);
        if (hipGetLastError() != hipSuccess) { set_error("k_bias_relu launch failed"); return SNAKE_E_LAUNCH; }
    }
    return SNAKE_OK;
}
