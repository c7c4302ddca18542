// Single-wave latency microbenchmarks for the reset worker's instruction mix
// (gfx950): cycles per iteration of dependent chains, measured with s_memtime.
//   hipcc --offload-arch=gfx950 -O3 -o lat lat.hip && ./lat
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int kIters = 4096;

__device__ __forceinline__ int mbcnt64(unsigned long long x)
{
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(x >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)x, 0u));
}

template <int P>
__global__ void k(unsigned long long *out, int *sink, int seed)
{
    const int lane = threadIdx.x;
    __shared__ unsigned lds[4096];
    for (int x = lane; x < 4096; x += 64) lds[x] = 0xffffffffu;
    __syncthreads();
    int v = lane * 7 + seed, acc = 0;
    unsigned long long m = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIters; it++) {
        if (P == 0) {                      // loop overhead only
            acc += it;
            __asm__ volatile("" : "+s"(acc));
        } else if (P == 1) {               // VALU -> ballot -> SALU popcount -> VALU (one round trip)
            m = __ballot(v <= acc);
            acc += __popcll(m);
            v += acc & 3;
        } else if (P == 2) {               // mbcnt chain on a ballot
            m = __ballot(v <= acc);
            v = v + mbcnt64(m);
            acc += 1;
        } else if (P == 3) {               // ds_min no-return x2 (fire and forget)
            __hip_atomic_fetch_min((__attribute__((address_space(3))) unsigned *)(lds + ((v * 13 + it) & 4095)),
                                   (unsigned)it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_min((__attribute__((address_space(3))) unsigned *)(lds + ((v * 29 + it) & 4095)),
                                   (unsigned)it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            v += 1;
        } else if (P == 4) {               // readfirstlane round trip
            acc += __builtin_amdgcn_readfirstlane(v);
            v += acc & 1;
        } else if (P == 5) {               // data-dependent uniform branch each iteration
            m = __ballot(v <= acc);
            if (m & 1ull) { acc += 3; } else { acc -= 1; }
            v += 1;
        } else if (P == 6) {               // LDS read dependent chain
            v = (int)lds[(v + it) & 4095] & 7;
            acc += v;
        } else if (P == 8) {               // 8 dependent SALU adds
            int x = acc;
#pragma unroll
            for (int r = 0; r < 8; r++) { x = x * 3 + it; __asm__ volatile("" : "+s"(x)); }
            acc = x;
        } else if (P == 9) {               // 8 dependent VALU ops
#pragma unroll
            for (int r = 0; r < 8; r++) { v = v * 3 + it; __asm__ volatile("" : "+v"(v)); }
        } else if (P == 10) {              // 8 independent VALU ops (4 chains of 2)
            int a = v, b = v + 1, c2 = v + 2, d = v + 3;
            a = a * 3 + it; b = b * 5 + it; c2 = c2 * 7 + it; d = d * 9 + it;
            __asm__ volatile("" : "+v"(a), "+v"(b), "+v"(c2), "+v"(d));
            a = a * 3 + 1; b = b * 5 + 1; c2 = c2 * 7 + 1; d = d * 9 + 1;
            __asm__ volatile("" : "+v"(a), "+v"(b), "+v"(c2), "+v"(d));
            v = a ^ b ^ c2 ^ d;
        } else if (P == 11) {              // ballot feeding only SALU (no VALU dependency back)
            m = __ballot(v <= it);
            acc += __popcll(m);
            v += 1;
        } else if (P == 12) {              // VALU op reading SGPR written by SALU each iter
            acc = acc * 5 + it;
            __asm__ volatile("" : "+s"(acc));
            v = v + acc;
            __asm__ volatile("" : "+v"(v));
        } else if (P == 7) {               // 4 independent ballots + SALU combine (refine-pass shape)
            const unsigned long long a = __ballot(v <= acc), b = __ballot(v <= acc + 5);
            const unsigned long long c = __ballot(v + 1 <= acc), d = __ballot(v + 2 <= acc);
            acc += (int)((a ^ b) | (c ^ d)) & 1;
            v += mbcnt64(a) + mbcnt64(c);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[0] = t1 - t0;
    sink[lane] = v + acc + (int)m;
}

template <int P>
double run(const char *name)
{
    unsigned long long *d_out;
    int *d_sink;
    hipMalloc(&d_out, 8);
    hipMalloc(&d_sink, 256);
    double best = 1e30;
    for (int r = 0; r < 5; r++) {
        hipLaunchKernelGGL(k<P>, dim3(1), dim3(64), 0, 0, d_out, d_sink, r);
        unsigned long long h = 0;
        hipMemcpy(&h, d_out, 8, hipMemcpyDeviceToHost);
        best = std::min(best, (double)h / kIters);
    }
    printf("%-50s %7.1f cycles/iter\n", name, best);
    hipFree(d_out);
    hipFree(d_sink);
    return best;
}

int main()
{
    run<0>("loop overhead");
    run<1>("ballot -> s_bcnt1 -> VALU round trip");
    run<2>("ballot -> mbcnt lo/hi -> VALU");
    run<3>("2x ds_min_u32 no-return (random addr)");
    run<4>("readfirstlane -> SALU -> VALU");
    run<5>("ballot -> uniform branch");
    run<6>("dependent ds_read_b32 chain");
    run<7>("4 ballots + SALU combine + 2 mbcnt");
    run<8>("8 dependent SALU mul-add");
    run<9>("8 dependent VALU mul-add");
    run<10>("8 independent VALU mul-add (4 chains)");
    run<11>("ballot -> SALU only");
    run<12>("SALU -> VALU reading it");
    return 0;
}
