// dqn32_kernels.hip -- the fp32 mode of the fused consumer: the reference's DQN
// forward (train_dqn.py:104-151) in fp32 arithmetic on any observation size,
// including train_dqn.py's own 20x20 full-map Config (:29-33).
//
// Every layer is one launch of k_gemm32, a 128x64-tile fp32 GEMM on the vector
// ALUs (gfx950's fp32 vector and fp32 matrix peaks are the same, 157 TF, and the
// vector form keeps the accumulation in plain fp32 FMAs):
//
//   Y[m][n] = sum_k act(X)[m][k] * W[n][k]          (W row-major [N][K])
//
// where the A operand is gathered on the fly (no im2col buffer):
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
    // conv1: uint8 NHWC obs -> Y1 [B*P][32]
    g.x = obs; g.xbias = nullptr; g.w = net->conv1_w; g.y = sc.y1; g.ybias = nullptr;
    g.M = BP; g.N = 32; g.K = 9 * C; g.C = C; g.scale_flag = sc.flag;
    if ((rc = dqn32::gemm<dqn32::kConvU8>(g, s, "conv1"))) return rc;
    // conv2: relu(Y1 + b1) -> Y2 [B*P][64]
    g.x = sc.y1; g.xbias = net->conv1_b; g.w = net->conv2_w; g.y = sc.y2;
    g.N = 64; g.K = 9 * 32; g.C = 32;
    if ((rc = dqn32::gemm<dqn32::kConvF32>(g, s, "conv2"))) return rc;
    // conv3: relu(Y2 + b2) -> Y3
    g.x = sc.y2; g.xbias = net->conv2_b; g.w = net->conv3_w; g.y = sc.y3;
    g.N = 64; g.K = 9 * 64; g.C = 64;
    if ((rc = dqn32::gemm<dqn32::kConvF32>(g, s, "conv3"))) return rc;
    // fc1: relu(Y3 + b3) flattened NHWC (P*64) -> Y4 [B][256]
    g.x = sc.y3; g.xbias = net->conv3_b; g.bmod = 64; g.w = net->fc1_w; g.y = sc.y4;
    g.M = batch; g.N = 256; g.K = (int)(P * 64);
    if ((rc = dqn32::gemm<dqn32::kDense>(g, s, "fc1"))) return rc;
    // fc2: relu(Y4 + bfc1) -> Y5 [B][128]
    g.x = sc.y4; g.xbias = net->fc1_b; g.bmod = 256; g.w = net->fc2_w; g.y = sc.y5;
    g.N = 128; g.K = 256;
    if ((rc = dqn32::gemm<dqn32::kDense>(g, s, "fc2"))) return rc;
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
