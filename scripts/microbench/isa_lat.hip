// Single-wave instruction-latency probes on gfx950 (cycles per repeated unit,
// s_memtime around 256 unrolled repeats). Informs the draw-round design of
// snake_kernels.hip (the permutation draws are one wave's dependency chain).
//   hipcc --offload-arch=gfx950 -O3 -o isa_lat isa_lat.hip && ./isa_lat
#include <hip/hip_runtime.h>
#include <stdio.h>

#define REP16(x) x x x x x x x x x x x x x x x x
#define REP256(x) REP16(REP16(x))

#define PROBE(name, setup, body)                                                      \
    __global__ void name(unsigned long long *out, int seed)                           \
    {                                                                                 \
        unsigned long long t0, t1;                                                    \
        int v0 = threadIdx.x + seed, v1 = seed * 3 + 1;                               \
        int s0 = seed;                                                                \
        unsigned long long sm = 0x5555ull + seed;                                     \
        setup;                                                                        \
        t0 = __builtin_amdgcn_s_memtime();                                            \
        __asm__ volatile("s_waitcnt lgkmcnt(0)\n" REP256(body)                         \
                         "s_waitcnt lgkmcnt(0)\n"                                     \
                         : "+v"(v0), "+v"(v1), "+s"(s0), "+s"(sm)::"vcc", "scc");      \
        t1 = __builtin_amdgcn_s_memtime();                                            \
        if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = (unsigned)v0 + s0 + sm; }  \
    }

// dependent VALU chain
PROBE(p_valu_dep, , "v_add_u32 %0, %0, %1\n")
// independent VALU (alternating registers)
PROBE(p_valu_indep, , "v_add_u32 %0, %0, 1\n v_add_u32 %1, %1, 1\n")
// dependent SALU chain
PROBE(p_salu_dep, , "s_add_u32 %2, %2, 1\n")
// VALU compare -> SALU use of the mask (dependent both ways via s0 operand)
PROBE(p_cmp_salu, , "v_cmp_gt_i32 vcc, %2, %0\n s_and_b64 %3, vcc, %3\n s_bcnt1_i32_b64 %2, %3\n")
// ballot -> mbcnt (SGPR written by SALU read by VALU) -> compare
PROBE(p_mbcnt_chain, ,
      "v_cmp_gt_i32 vcc, %1, %0\n s_and_b64 vcc, vcc, %3\n v_mbcnt_lo_u32_b32 %1, vcc_lo, 0\n v_mbcnt_hi_u32_b32 %1, vcc_hi, %1\n")
// VALU cmp -> VALU mbcnt reading the VALU-written VCC directly
PROBE(p_cmp_mbcnt, ,
      "v_cmp_gt_i32 vcc, %1, %0\n v_mbcnt_lo_u32_b32 %1, vcc_lo, 0\n v_mbcnt_hi_u32_b32 %1, vcc_hi, %1\n")
// taken forward branch
PROBE(p_branch, , "s_branch 1f\n s_nop 0\n 1:\n")
// not-taken conditional branch
PROBE(p_nobranch, , "s_cmp_eq_u32 %2, 12345677\n s_cbranch_scc1 1f\n 1:\n")
// taken conditional branch on scc
PROBE(p_cbranch, , "s_cmp_lg_u32 %2, 12345677\n s_cbranch_scc1 1f\n s_nop 0\n 1:\n")
// readlane with an SGPR-computed lane
PROBE(p_readlane, , "s_and_b32 %2, %2, 63\n v_readlane_b32 %2, %0, %2\n")
// ds_write_b16 stream (no wait), odd (misaligned) byte addresses
PROBE(p_dswrite, , "ds_write_b16 %0, %1\n")
// aligned ds_write_b16 / b32 (address 2*lane / 4*lane)
PROBE(p_dswrite16a, v0 = 2 * threadIdx.x, "ds_write_b16 %0, %1\n")
PROBE(p_dswrite32a, v0 = 4 * threadIdx.x, "ds_write_b32 %0, %1\n")
// aligned b16 with 2 independent VALU between
PROBE(p_dswrite16v, v0 = 2 * threadIdx.x, "ds_write_b16 %0, %1\n v_add_u32 %1, %1, 1\n v_xor_b32 %1, %1, 3\n")
// the same b16 address for all lanes (conflict)
PROBE(p_dswrite16s, v0 = 0, "ds_write_b16 %0, %1\n")

int main()
{
    unsigned long long *d, h[2];
    hipMalloc(&d, 16);
    struct { const char *n; void (*k)(unsigned long long *, int); int units; } ps[] = {
        {"valu dep (per instr)", p_valu_dep, 256},
        {"valu indep (per instr)", p_valu_indep, 512},
        {"salu dep (per instr)", p_salu_dep, 256},
        {"cmp->s_and->s_bcnt (per 3)", p_cmp_salu, 256},
        {"cmp->s_and->mbcnt lo/hi (per 4)", p_mbcnt_chain, 256},
        {"cmp->mbcnt lo/hi (per 3)", p_cmp_mbcnt, 256},
        {"s_branch taken (per)", p_branch, 256},
        {"s_cbranch not taken (per cmp+br)", p_nobranch, 256},
        {"s_cbranch taken (per cmp+br)", p_cbranch, 256},
        {"s_and->readlane (per 2)", p_readlane, 256},
        {"ds_write_b16 misaligned (per)", p_dswrite, 256},
        {"ds_write_b16 aligned (per)", p_dswrite16a, 256},
        {"ds_write_b32 aligned (per)", p_dswrite32a, 256},
        {"ds_write_b16 + 2 valu (per 3)", p_dswrite16v, 256},
        {"ds_write_b16 same addr (per)", p_dswrite16s, 256},
    };
    for (auto &p : ps) {
        unsigned long long best = ~0ull;
        for (int r = 0; r < 5; r++) {
            hipLaunchKernelGGL(p.k, dim3(1), dim3(64), 1024, 0, d, r);
            hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
            if (h[0] < best) best = h[0];
        }
        printf("%-36s %7.2f cycles\n", p.n, (double)best / p.units);
    }
    return 0;
}
