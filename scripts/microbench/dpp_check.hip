// Checks the DPP lane-group exchanges of snake_kernels.hip (gsel, gscan) against
// their definitions on random values: prints "dpp ok" or the first mismatches.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -I. dpp_check.hip -o dpp_check
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <utility>
#include <type_traits>
#include <stdint.h>

__device__ __forceinline__ int dpp_pin(int x) { __asm__ volatile("" : "+v"(x)); return x; }
template <int G, int J>
__device__ __forceinline__ int gsel(int v)
{
    if constexpr (G == 4) {
        return dpp_pin(__builtin_amdgcn_mov_dpp(v, J * 0x55, 0xf, 0xf, false));
    } else if constexpr (G == 16) {
        return dpp_pin(__builtin_amdgcn_mov_dpp(v, 0x150 + J, 0xf, 0xf, false));
    } else {
        const int t = dpp_pin(__builtin_amdgcn_mov_dpp(v, (J & 3) * 0x55, 0xf, 0xf, false));
        if constexpr (J < 4) return dpp_pin(__builtin_amdgcn_update_dpp(t, t, 0x114, 0xf, 0xa, false));
        else return dpp_pin(__builtin_amdgcn_update_dpp(t, t, 0x104, 0xf, 0x5, false));
    }
}
template <int G>
__device__ __forceinline__ int gscan(int v, int k)
{
    int x = dpp_pin(__builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false));
    v += k >= 1 ? x : 0;
    x = dpp_pin(__builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false));
    v += k >= 2 ? x : 0;
    if constexpr (G >= 8) { x = dpp_pin(__builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false)); v += k >= 4 ? x : 0; }
    if constexpr (G >= 16) { x = dpp_pin(__builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false)); v += k >= 8 ? x : 0; }
    return v;
}
// the same exchanges under a divergent branch in the caller (must still be right
// for the lanes that take it, reading lanes that do not)
template <typename F, int... I>
__device__ __forceinline__ void unroll_seq(F &&f, std::integer_sequence<int, I...>) { (f(std::integral_constant<int, I>{}), ...); }
template <int N, typename F>
__device__ __forceinline__ void unroll(F &&f) { unroll_seq(f, std::make_integer_sequence<int, N>{}); }

template <int G>
__global__ void k(const int *in, int *out)
{
    const int lane = threadIdx.x, k = lane % G;
    const int v = in[lane];
    unroll<G>([&](auto J) { out[J * 64 + lane] = gsel<G, J>(v); });
    out[G * 64 + lane] = gscan<G>(v, k);
}

template <int G>
int check(const int *din, int *dout, const int *hin)
{
    int h[17 * 64];
    hipLaunchKernelGGL(k<G>, dim3(1), dim3(64), 0, 0, din, dout);
    hipMemcpy(h, dout, sizeof(int) * (G + 1) * 64, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; l++) {
        const int gb = l / G * G;
        for (int j = 0; j < G; j++)
            if (h[j * 64 + l] != hin[gb + j]) { if (bad++ < 5) printf("G=%d gsel J=%d lane %d: %d != %d\n", G, j, l, h[j * 64 + l], hin[gb + j]); }
        int s = 0;
        for (int j = gb; j <= l; j++) s += hin[j];
        if (h[G * 64 + l] != s) { if (bad++ < 5) printf("G=%d gscan lane %d: %d != %d\n", G, l, h[G * 64 + l], s); }
    }
    return bad;
}

int main()
{
    int hin[64];
    srand(1);
    for (int i = 0; i < 64; i++) hin[i] = rand() % 1000 - 300;
    int *din, *dout;
    hipMalloc(&din, 64 * 4);
    hipMalloc(&dout, 17 * 64 * 4);
    hipMemcpy(din, hin, 64 * 4, hipMemcpyHostToDevice);
    const int bad = check<4>(din, dout, hin) + check<8>(din, dout, hin) + check<16>(din, dout, hin);
    printf(bad ? "dpp MISMATCH %d\n" : "dpp ok\n", bad);
    return bad != 0;
}
