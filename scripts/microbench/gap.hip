// Dependent-launch gap on one stream vs the bytes the first kernel leaves in L2
// (gfx950). Each case runs 200 x (writer; empty) back to back; time per pair from
// hipEvents minus the writer alone gives the gap the empty kernel adds.
//   hipcc --offload-arch=gfx950 -O3 -o gap gap.hip && ./gap
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int MODE>
__global__ void writer(uint4 *p, long long n16)
{
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long x = i; x < n16; x += stride) {
        uint4 v = make_uint4((unsigned)x, 1u, 2u, 3u);
        if (MODE == 0) p[x] = v;
        else if (MODE == 1) __builtin_nontemporal_store(v.x, &p[x].x), __builtin_nontemporal_store(v.y, &p[x].y),
                            __builtin_nontemporal_store(v.z, &p[x].z), __builtin_nontemporal_store(v.w, &p[x].w);
        else __hip_atomic_store(&p[x].x, v.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__global__ void empty_k(int *q) { if (threadIdx.x == 9999) q[0] = 1; }

template <int MODE>
static float run(uint4 *p, long long bytes, bool with_empty, int *q)
{
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    const long long n16 = bytes / 16;
    const int blocks = 2048;
    for (int w = 0; w < 20; w++) { writer<MODE><<<blocks, 256>>>(p, n16); if (with_empty) empty_k<<<1, 64>>>(q); }
    hipEventRecord(a);
    for (int w = 0; w < 200; w++) { writer<MODE><<<blocks, 256>>>(p, n16); if (with_empty) empty_k<<<1, 64>>>(q); }
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms * 1000.f / 200.f;
}

int main()
{
    uint4 *p; int *q;
    hipMalloc(&p, 256ll << 20); hipMalloc(&q, 4);
    const long long sizes[] = {0, 1 << 20, 8 << 20, 32 << 20, 64 << 20, 128 << 20, 256 << 20};
    for (long long s : sizes) {
        for (int mode = 0; mode < 3; mode++) {
            float solo, pair;
            if (mode == 0) { solo = run<0>(p, s, false, q); pair = run<0>(p, s, true, q); }
            else if (mode == 1) { solo = run<1>(p, s, false, q); pair = run<1>(p, s, true, q); }
            else { if (s > (64 << 20)) continue; solo = run<2>(p, s, false, q); pair = run<2>(p, s, true, q); }
            printf("{\"MB\": %lld, \"mode\": \"%s\", \"writer_us\": %.2f, \"pair_us\": %.2f, \"gap_us\": %.2f}\n",
                   s >> 20, mode == 0 ? "plain" : (mode == 1 ? "nt" : "sc1-dword"), solo, pair, pair - solo);
        }
    }
    return 0;
}
