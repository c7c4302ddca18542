// Cost of the step's fork/join between two streams of one device (gfx950):
// per-iteration time of 200 iterations of a k_logic-like writer (48 MB) followed
// by two kernels that should overlap, with different ways to order them.
//   hipcc --offload-arch=gfx950 -O3 -o forkjoin forkjoin.hip && ./forkjoin
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void writer(uint4 *p, long long n16, int tag)
{
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long x = i; x < n16; x += stride) p[x] = make_uint4((unsigned)x, tag, 2u, 3u);
}

// a fixed-duration kernel: one wave per block spins for `cycles`
__global__ void spin(long long cycles, int *sink)
{
    const long long t0 = clock64();
    while (clock64() - t0 < cycles) {}
    if (threadIdx.x == 9999) sink[0] = 1;
}

enum Mode { SERIAL, MARKER_ONLY, EVENTS, EVENTS_NOFENCE, WRITEWAIT };

static float run(Mode mode, uint4 *p, long long n16, int *sink, unsigned *flag, hipStream_t sm, hipStream_t ss)
{
    hipEvent_t fork, join, a, b;
    const unsigned fl = (mode == EVENTS_NOFENCE) ? (hipEventDisableTiming | hipEventDisableSystemFence)
                                                 : hipEventDisableTiming;
    hipEventCreateWithFlags(&fork, fl); hipEventCreateWithFlags(&join, fl);
    hipEventCreate(&a); hipEventCreate(&b);
    const long long spin_long = 100000, spin_short = 50000;   // ~40 / ~20 us at ~2.4 GHz
    auto iter = [&](int it) {
        writer<<<2048, 256, 0, sm>>>(p, n16, it);
        if (mode == SERIAL) {
            spin<<<256, 64, 0, sm>>>(spin_long, sink);
            spin<<<256, 64, 0, sm>>>(spin_short, sink);
        } else if (mode == MARKER_ONLY) {
            hipEventRecord(fork, sm);
            spin<<<256, 64, 0, sm>>>(spin_long, sink);
            spin<<<256, 64, 0, sm>>>(spin_short, sink);
        } else if (mode == EVENTS || mode == EVENTS_NOFENCE) {
            hipEventRecord(fork, sm);
            hipStreamWaitEvent(ss, fork, 0);
            spin<<<256, 64, 0, sm>>>(spin_long, sink);
            spin<<<256, 64, 0, ss>>>(spin_short, sink);
            hipEventRecord(join, ss);
            hipStreamWaitEvent(sm, join, 0);
        } else {
            hipStreamWriteValue32(sm, flag, (uint32_t)(2 * it + 1), 0);
            hipStreamWaitValue32(ss, flag, (uint32_t)(2 * it + 1), hipStreamWaitValueGte, 0xffffffffu);
            spin<<<256, 64, 0, sm>>>(spin_long, sink);
            spin<<<256, 64, 0, ss>>>(spin_short, sink);
            hipStreamWriteValue32(ss, flag + 1, (uint32_t)(2 * it + 2), 0);
            hipStreamWaitValue32(sm, flag + 1, (uint32_t)(2 * it + 2), hipStreamWaitValueGte, 0xffffffffu);
        }
    };
    static int base = 0;
    for (int w = 0; w < 20; w++) iter(base++);
    hipEventRecord(a, sm);
    for (int w = 0; w < 200; w++) iter(base++);
    hipEventRecord(b, sm);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms * 1000.f / 200.f;
}

int main()
{
    uint4 *p; int *sink; unsigned *flag;
    hipMalloc(&p, 64ll << 20); hipMalloc(&sink, 4);
    hipExtMallocWithFlags((void **)&flag, 64, hipMallocSignalMemory);
    hipMemset(flag, 0, 64);
    hipStream_t sm, ss;
    hipStreamCreateWithFlags(&sm, hipStreamNonBlocking);
    hipStreamCreateWithFlags(&ss, hipStreamNonBlocking);
    const long long n16 = (48ll << 20) / 16;
    const char *names[] = {"serial", "marker_only", "events", "events_nofence", "write_wait_value"};
    for (int rep = 0; rep < 2; rep++)
        for (int m = 0; m < 5; m++)
            printf("{\"mode\": \"%s\", \"us_per_iter\": %.2f}\n", names[m],
                   run((Mode)m, p, n16, sink, flag, sm, ss));
    return 0;
}
