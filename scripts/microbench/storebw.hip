// Store-bandwidth probe for the observation write (k_post's encodes): every
// wave writes EPW consecutive envs of `env_bytes` (3 872 at cfg3) as 16-byte
// stores (1 KB per wave-instruction), optionally non-temporal, optionally with
// dynamic LDS per block (to cap occupancy like k_post's 8.1 KB) and a delay
// between envs (an env's lookups). Compares with a grid-stride store kernel.
//   hipcc -O3 --offload-arch=gfx950 -o storebw storebw.hip && ./storebw
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ void k_env_stores(uint8_t *out, int n_env, int env_bytes, int epw, int spin)
{
    extern __shared__ uint8_t lds[];
    const int lane = threadIdx.x & 63;
    const int wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int chunks = env_bytes / 16;
    if (blockDim.x == 64) lds[lane] = (uint8_t)lane;
    for (int q = 0; q < epw; q++) {
        const int e = wave * epw + q;
        if (e >= n_env) break;
        v4u *o = reinterpret_cast<v4u *>(out + (int64_t)e * env_bytes);
        unsigned long long t0 = __builtin_amdgcn_s_memtime();
        while (spin && __builtin_amdgcn_s_memtime() - t0 < (unsigned long long)spin) {}
        for (int c = lane; c < chunks; c += 64) {
            const v4u v = (v4u){(uint32_t)e, (uint32_t)c, 1u, 2u};
            if (NT) __builtin_nontemporal_store(v, o + c);
            else o[c] = v;
        }
    }
}

__global__ void k_stride_stores(v4u *out, int64_t n16)
{
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x)
        __builtin_nontemporal_store((v4u){1u, 2u, 3u, (uint32_t)i}, out + i);
}

int main()
{
    const int n_env = 65536, env_bytes = 3872;
    const int64_t bytes = (int64_t)n_env * env_bytes;
    // four buffers written in turn (1 GB: no reuse from the 256 MB Infinity Cache)
    uint8_t *buf;
    (void)hipMalloc(&buf, 4 * bytes + 4096);
    int it = 0;
    uint8_t *out = buf;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto timeit = [&](const char *name, auto launch0) {
        auto launch = [&]() { out = buf + (int64_t)(it++ & 3) * bytes; launch0(); };
        for (int i = 0; i < 3; i++) launch();
        hipDeviceSynchronize();
        const int R = 20;
        hipEventRecord(a);
        for (int i = 0; i < R; i++) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        ms /= R;
        printf("%-48s %8.2f us  %6.2f TB/s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
    };
    for (int nt = 0; nt < 2; nt++)
        for (int epw : {1, 4, 16})
            for (int lds : {0, 8192})
                for (int spin : {0, 2000}) {
                    char nm[128];
                    snprintf(nm, sizeof nm, "env stores %s epw %2d lds %5d spin %4d", nt ? "nt " : "wb ", epw, lds, spin);
                    const int waves = (n_env + epw - 1) / epw;
                    timeit(nm, [&]() {
                        if (nt) hipLaunchKernelGGL(k_env_stores<true>, dim3(waves), dim3(64), lds, 0, out, n_env, env_bytes, epw, spin);
                        else hipLaunchKernelGGL(k_env_stores<false>, dim3(waves), dim3(64), lds, 0, out, n_env, env_bytes, epw, spin);
                    });
                }
    timeit("grid-stride nt, 2048 x 256", [&]() {
        hipLaunchKernelGGL(k_stride_stores, dim3(2048), dim3(256), 0, 0, (v4u *)out, bytes / 16);
    });
    timeit("grid-stride nt, 8192 x 256", [&]() {
        hipLaunchKernelGGL(k_stride_stores, dim3(8192), dim3(256), 0, 0, (v4u *)out, bytes / 16);
    });
    (void)hipFree(buf);
    return 0;
}
