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

constexpr int kMaxMt = 9;         // position tiles of 16: h*w <= 144 (vision_range <= 5)
constexpr int kFcObs = 128;       // observations per k_dqn_fc workgroup

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

// A fragment of the implicit GEMM: the 8 consecutive k = 8 channels of one tap
// (tap = k0 / CIN, channels k0 % CIN ..) at output position p, from the NHWC
// bf16 image src[P16][CIN]; zero for a padding row, a tap past the 9th or a
// source position off the map (the convolution's zero padding).
template <int CINL>
__device__ __forceinline__ bf16x8 gather(const uint16_t *src, int p, int k0, int P, int H, int W, uint32_t magW)
{
    constexpr int CIN = 1 << CINL;
    const int tap = k0 >> CINL, ci = k0 & (CIN - 1);
    const int y = (int)__umulhi((uint32_t)p, magW), x = p - y * W;
    const int ty = tap >= 6 ? 2 : (tap >= 3 ? 1 : 0);
    const int yy = y + ty - 1, xx = x + (tap - 3 * ty) - 1;
    const bool ok = tap < 9 && p < P && (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
    const int q = ok ? (yy * W + xx) * CIN + ci : 0;
    const bf16x8 v = *reinterpret_cast<const bf16x8 *>(src + q);
    return ok ? v : (bf16x8)0;
}

// One 3x3 convolution + bias + ReLU of the wave's observation: src NHWC bf16
// [P16][CIN] in LDS -> dst NHWC bf16 [P16][COUT] in LDS, or (gdst) NCHW bf16
// [COUT][P16] in global memory. wt = [COUT][K] bf16, K = ksteps * 32.
template <int CINL, int COUT>
__device__ void conv_layer(const uint16_t *src, uint16_t *dst, uint16_t *gdst, const uint16_t *__restrict__ wt,
                           const float *__restrict__ bias, int ksteps, int MT, int P, int H, int W,
                           uint32_t magW, int lane)
{
    const int r16 = lane & 15, kq = 8 * (lane >> 4);
    const int K = ksteps * 32;
    for (int nt = 0; nt < COUT / 16; nt++) {
        f32x4 acc[kMaxMt];
#pragma unroll
        for (int m = 0; m < kMaxMt; m++) acc[m] = (f32x4)0.0f;
        const uint16_t *wrow = wt + (int64_t)(nt * 16 + r16) * K + kq;
        for (int ks = 0; ks < ksteps; ks++) {
            const bf16x8 b = *reinterpret_cast<const bf16x8 *>(wrow + ks * 32);
            const int k0 = ks * 32 + kq;
#pragma unroll
            for (int m = 0; m < kMaxMt; m++) {
                if (m < MT) {
                    const bf16x8 a = gather<CINL>(src, m * 16 + r16, k0, P, H, W, magW);
                    acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[m], 0, 0, 0);
                }
            }
        }
        // D[row (lane >> 4) * 4 + r][col lane & 15]: 4 positions of one channel
        const int co = nt * 16 + r16;
        const float bb = bias[co];
#pragma unroll
        for (int m = 0; m < kMaxMt; m++) {
            if (m < MT) {
                const int p0 = m * 16 + 4 * (lane >> 4);
                uint32_t v[4];
#pragma unroll
                for (int r = 0; r < 4; r++) v[r] = bf16_bits(fmaxf(acc[m][r] + bb, 0.0f));
                if (dst) {
#pragma unroll
                    for (int r = 0; r < 4; r++) dst[(p0 + r) * COUT + co] = (uint16_t)v[r];
                } else {
                    uint2 w2;
                    w2.x = v[0] | (v[1] << 16);
                    w2.y = v[2] | (v[3] << 16);
                    *reinterpret_cast<uint2 *>(gdst + (int64_t)co * (MT * 16) + p0) = w2;
                }
            }
        }
    }
}

struct ConvArgs {
    const uint8_t *obs;
    int64_t B;
    int H, W, C, CL, P, MT, k1steps;   // CL = log2 of the padded input channels
    uint32_t magW;
    const uint16_t *w1, *w2, *w3;
    const float *b1, *b2, *b3;
    uint16_t *act;                      // [B][64][MT*16]
};

template <int CL>
__global__ void __launch_bounds__(64) k_dqn_conv(const ConvArgs a)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int lane = threadIdx.x;
    const int P16 = a.MT * 16, CP = 1 << CL;
    uint16_t *a0 = reinterpret_cast<uint16_t *>(lds);   // [P16][CP]
    uint16_t *a1 = a0 + P16 * CP;                        // [P16][32]
    uint16_t *a2 = a1 + P16 * 32;                        // [P16][64]
    for (int64_t b = blockIdx.x; b < a.B; b += gridDim.x) {
        // x.permute(0, 3, 1, 2).float(): the NHWC bytes, as bf16 (0/1 exact),
        // padded to CP channels and P16 positions with zeros
        const uint8_t *x = a.obs + b * (int64_t)a.P * a.C;
        for (int i = lane; i < P16 * CP; i += 64) {
            const int p = i >> CL, ch = i & (CP - 1);
            const int v = (p < a.P && ch < a.C) ? x[p * a.C + ch] : 0;
            a0[i] = (uint16_t)bf16_bits((float)v);
        }
        wave_lds_sync();
        conv_layer<CL, 32>(a0, a1, nullptr, a.w1, a.b1, a.k1steps, a.MT, a.P, a.H, a.W, a.magW, lane);
        wave_lds_sync();
        conv_layer<5, 64>(a1, a2, nullptr, a.w2, a.b2, 9, a.MT, a.P, a.H, a.W, a.magW, lane);
        wave_lds_sync();
        conv_layer<6, 64>(a2, nullptr, a.act + b * 64 * P16, a.w3, a.b3, 18, a.MT, a.P, a.H, a.W, a.magW, lane);
        wave_lds_sync();
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

__global__ void __launch_bounds__(512) k_dqn_fc(const FcArgs a)
{
    // fc1 weight k-step tiles (double buffered); afterwards the h1 / h2 slices of
    // four waves at a time (8 KB each)
    __shared__ __attribute__((aligned(16))) uint16_t bt[2][256 * 32];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int r16 = lane & 15, kq = 8 * (lane >> 4);
    const int64_t ob0 = (int64_t)blockIdx.x * kFcObs + wv * 16;   // this wave's 16 observations
    const int64_t orow = ob0 + r16;
    const bool rok = orow < a.B;
    const uint16_t *arow = a.act + (rok ? orow : 0) * (int64_t)a.K + kq;
    const int ksteps = a.K / 32;
    // the tile loader: thread t copies 16 k of fc1 row t/2 (one k step = 256 x 32)
    const int ln = tid >> 1, lh = (tid & 1) * 16;
    const uint16_t *wsrc = a.w4 + (int64_t)ln * a.K + lh;
    auto load_tile = [&](int ks, int buf) {
        const u32x4 *s = reinterpret_cast<const u32x4 *>(wsrc + ks * 32);
        u32x4 *d = reinterpret_cast<u32x4 *>(&bt[buf][ln * 32 + lh]);
        d[0] = s[0];
        d[1] = s[1];
    };
    f32x4 acc[16];
#pragma unroll
    for (int n = 0; n < 16; n++) acc[n] = (f32x4)0.0f;
    load_tile(0, 0);
    __syncthreads();
    for (int ks = 0; ks < ksteps; ks++) {
        const int buf = ks & 1;
        if (ks + 1 < ksteps) load_tile(ks + 1, buf ^ 1);
        bf16x8 av = *reinterpret_cast<const bf16x8 *>(arow + ks * 32);
        if (!rok) av = (bf16x8)0;
#pragma unroll
        for (int n = 0; n < 16; n++) {
            const bf16x8 bv = *reinterpret_cast<const bf16x8 *>(&bt[buf][(n * 16 + r16) * 32 + kq]);
            acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc[n], 0, 0, 0);
        }
        __syncthreads();
    }
    // fc2 and fc3, waves 0-3 then 4-7 (their h1 / h2 slices reuse the tile buffer)
    uint32_t *hbuf = reinterpret_cast<uint32_t *>(&bt[0][0]);
    for (int phase = 0; phase < 2; phase++) {
        if ((wv >> 2) == phase) {
            uint32_t *hw = hbuf + (wv & 3) * 2048;
            // h1 = relu(fc1 + b) as bf16 [16][256]
            uint16_t *h1 = reinterpret_cast<uint16_t *>(hw);
#pragma unroll
            for (int n = 0; n < 16; n++) {
                const int col = n * 16 + r16;
                const float bb = a.b4[col];
#pragma unroll
                for (int r = 0; r < 4; r++)
                    h1[(4 * (lane >> 4) + r) * 256 + col] = (uint16_t)bf16_bits(fmaxf(acc[n][r] + bb, 0.0f));
            }
            wave_lds_sync();
            // fc2: [16 x 256] x [256 x 128]
            f32x4 acc2[8];
#pragma unroll
            for (int n = 0; n < 8; n++) acc2[n] = (f32x4)0.0f;
#pragma unroll
            for (int ks = 0; ks < 8; ks++) {
                const bf16x8 av = *reinterpret_cast<const bf16x8 *>(&h1[r16 * 256 + ks * 32 + kq]);
#pragma unroll
                for (int n = 0; n < 8; n++) {
                    const bf16x8 bv =
                        *reinterpret_cast<const bf16x8 *>(a.w5 + (n * 16 + r16) * 256 + ks * 32 + kq);
                    acc2[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc2[n], 0, 0, 0);
                }
            }
            wave_lds_sync();
            // h2 = relu(fc2 + b) fp32 [16][128] (forward_features), then fc3 in fp32
            float *h2 = reinterpret_cast<float *>(hw);
#pragma unroll
            for (int n = 0; n < 8; n++) {
                const int col = n * 16 + r16;
                const float bb = a.b5[col];
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int row = 4 * (lane >> 4) + r;
                    const float v = fmaxf(acc2[n][r] + bb, 0.0f);
                    h2[row * 128 + col] = v;
                    if (a.feat && ob0 + row < a.B) a.feat[(ob0 + row) * 128 + col] = v;
                }
            }
            wave_lds_sync();
            if (lane < 16 * a.A) {
                const int row = lane / a.A, act = lane - row * a.A;
                float sum = a.b6[act];
                const float *w = a.w6 + act * 128;
                for (int k = 0; k < 128; k++) sum = fmaf(h2[row * 128 + k], w[k], sum);
                if (ob0 + row < a.B) a.q[(ob0 + row) * a.A + act] = sum;
            }
        }
        __syncthreads();
    }
}

}  // namespace dqn
}  // namespace snake

using namespace snake;
using namespace snake::dqn;

extern "C" int snake_dqn_plan(const snake_dqn_cfg *cfg, snake_dqn_layout *out)
{
    if (!cfg || !out) { set_error("snake_dqn_plan: NULL argument"); return SNAKE_E_ARG; }
    const int H = cfg->height, W = cfg->width, C = cfg->channels, A = cfg->num_actions;
    if (H < 1 || W < 1 || H * W > 16 * kMaxMt || W > 16) {
        set_error("snake_dqn: h*w must be <= %d and w <= 16 (vision_range <= 5), got %dx%d", 16 * kMaxMt, H, W);
        return SNAKE_E_CONFIG;
    }
    if (C < 1 || C > 32) { set_error("snake_dqn: channels must be in [1, 32] (got %d)", C); return SNAKE_E_CONFIG; }
    if (A < 1 || A > 4) { set_error("snake_dqn: num_actions must be in [1, 4] (got %d)", A); return SNAKE_E_CONFIG; }
    int cl = 3;
    while ((1 << cl) < C) cl++;
    const int MT = (H * W + 15) / 16, P16 = MT * 16, CP = 1 << cl;
    out->cpad = CP;
    out->p16 = P16;
    out->k1 = (9 * CP + 31) / 32 * 32;
    out->conv1_w = 32ll * out->k1;
    out->conv2_w = 64ll * 288;
    out->conv3_w = 64ll * 576;
    out->fc1_w = 256ll * 64 * P16;
    out->fc2_w = 128ll * 256;
    out->act_per_obs = 64ll * P16;
    out->lds_conv = (int32_t)(2 * P16 * (CP + 32 + 64));
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
    ca.obs = obs; ca.B = batch; ca.H = cfg->height; ca.W = cfg->width; ca.C = cfg->channels;
    ca.P = ca.H * ca.W; ca.MT = lay.p16 / 16; ca.k1steps = lay.k1 / 32;
    ca.CL = 3;
    while ((1 << ca.CL) < lay.cpad) ca.CL++;
    ca.magW = (uint32_t)(((1ull << 32) + ca.W - 1) / ca.W);
    ca.w1 = net->conv1_w; ca.w2 = net->conv2_w; ca.w3 = net->conv3_w;
    ca.b1 = net->conv1_b; ca.b2 = net->conv2_b; ca.b3 = net->conv3_b;
    ca.act = act_scratch;
    const unsigned gconv = (unsigned)std::min<int64_t>(batch, 256 * 24);
    if (ca.CL == 3) hipLaunchKernelGGL(k_dqn_conv<3>, dim3(gconv), dim3(64), lay.lds_conv, s, ca);
    else if (ca.CL == 4) hipLaunchKernelGGL(k_dqn_conv<4>, dim3(gconv), dim3(64), lay.lds_conv, s, ca);
    else hipLaunchKernelGGL(k_dqn_conv<5>, dim3(gconv), dim3(64), lay.lds_conv, s, ca);
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
