// snake_kernels.hip -- the batched multi-snake env step on CDNA4 (gfx950).
//
// snake_step = k_logic, then one shared-phase launch (k_post / k_post_lean:
// reset workers + encodes), with the spawn-ahead attempts in the step or in
// k_spawn on the library's background streams (launch_step):
//   * k_logic: 4, 8 or 16 lanes per env, the envs' current grids staged in LDS
//     with 16-byte loads; the game rules (snake_env.py:301-374) lane-parallel,
//     lane (env g, snake k): targets, collision groups (DPP moves inside the
//     env's lane group), the fruit-eater tail rule, rewards,
//     and a two-phase grid update (all tail clears, then all BODY/HEAD/TAIL
//     writes) that reproduces the reference's snake-order update exactly
//     ("two-phase update"); dead-body erase (prefix-scanned direction
//     deque), fruit respawn (lane-chunked empty-cell ranking + MT19937 rejection
//     sampling resolved by ballots); envs whose dones are all True are queued;
//   * encodes: the NHWC one-hot observation from the grid ring as table lookups
//     (encode_tbl_block), 16-byte non-temporal stores;
//   * reset workers / k_reset: in-register MT19937 twist, Fisher-Yates draws in
//     ballot-refined rounds recording the draws, trace of arr[:S], paint,
//     fruits, encode.
// Compiled with -ffp-contract=off: rewards/statistics are float64 in the
// reference's order of operations (snake_env.py:365-369, :385-389).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <limits.h>
#include <stdlib.h>
#include <string.h>

#include <map>
#include <string>
#include <vector>
#include <mutex>
#include <type_traits>
#include <utility>

#include "snake_internal.h"

constexpr int kResetWavesPerEU = 4;   // reset workers: 128 VGPRs (3 waves/SIMD measured slower)

namespace snake {

// Every launch goes through hipExtLaunchKernel: while a launch is timed
// (TimedLaunch, snake_timing_enable) these are its start/stop events, which then
// carry the dispatch's own begin/end timestamps -- no marker packets of their
// own between the step's kernels (hipEventRecord pairs left 6 + 10.5 us gaps
// around each timed step's k_logic / k_post in the kernel trace). Null: a
// plain launch.
thread_local hipEvent_t t_ev0 = nullptr, t_ev1 = nullptr;
template <typename F, typename... Args>
static inline void slaunch(F kernel, const dim3 &grid, const dim3 &block, uint32_t lds, hipStream_t s,
                           Args... args)
{
    hipExtLaunchKernelGGL(kernel, grid, block, lds, s, t_ev0, t_ev1, 0u, args...);
}

__device__ unsigned long long g_resets_run;     // auto-resets run (snake_timing_read "resets")
__device__ unsigned long long g_resets_timed;   // the same, while timing is enabled ("resets_timed")
// (diagnostic counters, spread over 64 lines by block: one address taking a
// device-scope atomic per job serialised thousands of them on the timed steps)
constexpr int kDiagSlots = 64, kDiagSpread = 16;
__device__ unsigned long long g_spawn_hits[kDiagSlots * kDiagSpread];   // auto-resets that found a ready record
__device__ unsigned long long g_spawn_jobs[kDiagSlots * kDiagSpread];   // spawn-ahead jobs dequeued
__device__ unsigned long long g_spawn_void[kDiagSlots * kDiagSpread];   // ready records voided by a fruit draw
__device__ unsigned long long g_reset_part[kDiagSlots * kDiagSpread];   // auto-resets that found a partial record
__device__ unsigned long long g_resp_slow[kDiagSlots * kDiagSpread];    // k_logic respawns on the full-wave path (no room)
__device__ unsigned long long g_resp_slow2[kDiagSlots * kDiagSpread];   // ... (room, too few accepts among the prefetched raws)
__device__ unsigned long long g_gate_shut[kDiagSlots * kDiagSpread];    // k_logic waves that found the background queue set busy
__device__ unsigned long long g_draw_wait[kDiagSlots * kDiagSpread];    // resets that waited for a background job (DRAWING)
__device__ unsigned long long g_draw_timeout[kDiagSlots * kDiagSpread]; // ... and gave up waiting (drew from the env's own state)
#define DIAG_ADD(arr) atomicAdd(&(arr)[(blockIdx.x % kDiagSlots) * kDiagSpread], 1ull)
#ifdef SNAKE_FUSE_DEBUG
// (diagnostic build: range checks on the fused step's indices; a violation is
// recorded -- site, value -- and the access skipped)
__device__ unsigned long long g_fdbg[64];
#define FDBG_BAD(site, val) (atomicAdd(&g_fdbg[2 * (site)], 1ull), atomicMax(&g_fdbg[2 * (site) + 1], (unsigned long long)(uint32_t)(val)), true)
#define FDBG_MARK(site) do { if ((threadIdx.x & 63) == 0) atomicAdd(&g_fdbg[2 * (site)], 1ull); } while (0)
#else
#define FDBG_BAD(site, val) false
#define FDBG_MARK(site) do {} while (0)
#endif

#ifdef SNAKE_STAMPS
// Diagnostic build only (scripts/logic_stamps.py): s_memtime stamps of block
// 0's wave at k_logic's phase boundaries, and s_memrealtime (100 MHz) at every
// k_logic wave's start and end (its block index, up to kWaveTimes blocks).
constexpr int kWaveTimes = 8192, kPostTimes = 40960;
__device__ unsigned long long g_stamps[64];
__device__ unsigned long long g_wavetime[2 * kWaveTimes];
__device__ unsigned long long g_posttime[2 * kPostTimes];   // k_post: every block's start and end
#define PTIME(end)                                                                 \
    do {                                                                           \
        __builtin_amdgcn_sched_barrier(0);                                         \
        if ((threadIdx.x & 63) == 0 && blockIdx.x < kPostTimes)                    \
            g_posttime[2 * blockIdx.x + (end)] = __builtin_amdgcn_s_memrealtime(); \
        __builtin_amdgcn_sched_barrier(0);                                         \
    } while (0)
// (and every k_logic wave's s_memrealtime at each phase: g_wphase[wave][idx - 40])
__device__ unsigned long long g_wphase[16 * kWaveTimes];
#define LSTAMP(idx)                                                                \
    do {                                                                           \
        __builtin_amdgcn_sched_barrier(0);                                         \
        if (blockIdx.x == 0) {                                                     \
            unsigned long long _t = __builtin_amdgcn_s_memtime();                  \
            if (threadIdx.x == 0) g_stamps[idx] = _t;                              \
        }                                                                          \
        const unsigned _w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);  \
        if ((threadIdx.x & 63) == 0 && _w < kWaveTimes)                            \
            g_wphase[16 * _w + (idx) - 40] = __builtin_amdgcn_s_memrealtime();     \
        __builtin_amdgcn_sched_barrier(0);                                         \
    } while (0)
#define WTIME(end)                                                                 \
    do {                                                                           \
        __builtin_amdgcn_sched_barrier(0);                                         \
        const unsigned _w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);  \
        if ((threadIdx.x & 63) == 0 && _w < kWaveTimes)                            \
            g_wavetime[2 * _w + (end)] = __builtin_amdgcn_s_memrealtime();         \
        __builtin_amdgcn_sched_barrier(0);                                         \
    } while (0)
// every reset-worker item (scripts/post_items.py): worker | type << 32, start,
// end (s_memrealtime), env; types 0 reset from a ready record, 1 from a partial
// one, 2 without one, 3 queue-1 spawn-ahead job, 4 queue-2 job
constexpr int kItems = 16384;
__device__ unsigned g_nitems;
__device__ unsigned long long g_items[4 * kItems];
#define ITEM_T0() const unsigned long long _it0 = __builtin_amdgcn_s_memrealtime()
#define ITEM_LOG(wid, type, e)                                                                      \
    do {                                                                                           \
        __builtin_amdgcn_sched_barrier(0);                                                         \
        const unsigned long long _it1 = __builtin_amdgcn_s_memrealtime();                          \
        if ((threadIdx.x & 63) == 0) {                                                             \
            const unsigned _i = atomicAdd(&g_nitems, 1u);                                          \
            if (_i < kItems) {                                                                     \
                g_items[4 * _i] = (unsigned long long)(wid) | ((unsigned long long)(type) << 32);   \
                g_items[4 * _i + 1] = _it0; g_items[4 * _i + 2] = _it1;                             \
                g_items[4 * _i + 3] = (unsigned long long)(e);                                     \
            }                                                                                      \
        }                                                                                          \
    } while (0)
#else
#define ITEM_T0() do {} while (0)
#define ITEM_LOG(wid, type, e) do {} while (0)
#define LSTAMP(idx) do {} while (0)
#define WTIME(end) do {} while (0)
#define PTIME(end) do {} while (0)
#endif

enum { C_EMPTY = 0, C_WALL = 1, C_FRUIT = 2, C_HEAD = 3, C_BODY = 4, C_TAIL = 5 };

// The step and reset kernels take their arguments as one struct and read them
// through kargs(): a pointer to the kernarg segment that the compiler cannot see
// through (an empty asm), taken afresh at each phase or job. Every field is then
// an s_load next to its use (the segment is constant, scalar-cached) instead of
// a value held in an SGPR from the kernel's entry to its end: with the whole
// KCfg, snake_state and snake_out live across a worker's job loop the compiler
// spilled 230-300 SGPRs into VGPR lanes, 1 100-1 700 v_readlane reloads and
// 128 VGPRs (profiles/r03_isa_counts.jsonl).
struct KArgs {
    KCfg c;
    snake_state st;
    snake_out o;
    const void *aux;   // k_logic: the actions; k_reset: the env mask
};

__device__ __forceinline__ const KArgs &kargs()
{
    typedef const __attribute__((address_space(4))) KArgs KA4;
    KA4 *p = (KA4 *)__builtin_amdgcn_kernarg_segment_ptr();   // (the first explicit argument is at offset 0)
    __asm__ volatile("" : "+s"(p));
    return *(const KArgs *)p;
}

// global-memory views (explicit address space: flat accesses would also count
// against lgkmcnt and stall every LDS/cross-lane wait behind them)
typedef __attribute__((address_space(3))) uint16_t lu16;
typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(3))) uint32_t lu32;
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) v4u32 gu4;
typedef __attribute__((address_space(3))) v4u32 lu4;
constexpr uint32_t kNoLink = 0xffffffffu;

// Link-table access: LDS atomics are ds_min_u32, global ones L2 atomics; global
// reads bypass the vector L1 (a previous attempt's chase may have cached lines).
__device__ __forceinline__ void link_min(lu32 *p, uint32_t v)
{
    __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void link_min(gu32 *p, uint32_t v)
{
    __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t link_get(const lu32 *p) { return *p; }
__device__ __forceinline__ uint32_t link_get(const gu32 *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A worker's global link table between its writers and its readers, all lanes
// of one wave: the wave's stores and atomics complete at device scope, then a
// wave barrier.
__device__ __forceinline__ void link_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
    __builtin_amdgcn_wave_barrier();
}

// Direction (core/snake.py:33-37): 0 UP(-1,0) 1 RIGHT(0,1) 2 DOWN(1,0) 3 LEFT(0,-1)
__device__ __forceinline__ int dir_dr(int d) { return d == 0 ? -1 : (d == 2 ? 1 : 0); }
__device__ __forceinline__ int dir_dc(int d) { return d == 1 ? 1 : (d == 3 ? -1 : 0); }
__device__ __forceinline__ int div10(int v) { return (v * 205) >> 11; }  // exact for 0 <= v < 1029
// x / d by the multiply-high reciprocal m = ceil(2^32 / d) (snake_capi.cpp);
// d == 1 has no 32-bit reciprocal (m wraps to 0)
__device__ __forceinline__ int fdiv(uint32_t x, uint32_t m, int d) { return d == 1 ? (int)x : (int)__umulhi(x, m); }

// LDS hand-off between lanes of the single wave of a workgroup: LDS executes a
// wave's instructions in order, so only the compiler must not move memory
// operations across this point.
__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ int wave_scan(int v, int lane)
{
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const int n = __shfl_up(v, o);
        if (lane >= o) v += n;
    }
    return v;
}

__device__ __forceinline__ int bcast(int v, int k) { return __builtin_amdgcn_readlane(v, k); }

// ---- exchanges inside k_logic's env groups of G = 4, 8 or 16 lanes (aligned
// inside a 16-lane DPP row) by DPP moves, not through the LDS: a __shfl
// (ds_bpermute) is an LDS round trip on the rules' dependency chain.
// A DPP move reads its source lane's register only when that lane is active:
// every move here runs with the whole wave active, and its result passes
// through an empty volatile asm, so the compiler cannot sink it into a branch
// that only some lanes take (it did: a select on a DPP result became an
// exec-masked branch around the move, which then read disabled lanes).
__device__ __forceinline__ int dpp_pin(int x)
{
    __asm__ volatile("" : "+v"(x));
    return x;
}

// gsel<G, J>(v): the value of lane J of this lane's group.
template <int G, int J>
__device__ __forceinline__ int gsel(int v)
{
    static_assert(G == 4 || G == 8 || G == 16, "group of 4, 8 or 16 lanes");
    if constexpr (G == 4) {
        return dpp_pin(__builtin_amdgcn_mov_dpp(v, J * 0x55, 0xf, 0xf, false));   // quad_perm:[J,J,J,J]
    } else if constexpr (G == 16) {
        return dpp_pin(__builtin_amdgcn_mov_dpp(v, 0x150 + J, 0xf, 0xf, false));   // row_newbcast:J
    } else {
        // lane J & 3 of the lane's quad; then the group's other quad (DPP banks
        // 1, 3 for J < 4, else 0, 2) takes that value from four lanes over,
        // the bank mask keeping the rest
        const int t = dpp_pin(__builtin_amdgcn_mov_dpp(v, (J & 3) * 0x55, 0xf, 0xf, false));
        if constexpr (J < 4) return dpp_pin(__builtin_amdgcn_update_dpp(t, t, 0x114, 0xf, 0xa, false));   // row_shr:4
        else return dpp_pin(__builtin_amdgcn_update_dpp(t, t, 0x104, 0xf, 0x5, false));                   // row_shl:4
    }
}

template <int G, int J>
__device__ __forceinline__ double gsel(double v)
{
    const long long b = __double_as_longlong(v);
    const int lo = gsel<G, J>((int)b), hi = gsel<G, J>((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (uint32_t)lo);
}

// inclusive prefix sum over the group (k = the lane's index in it)
template <int G>
__device__ __forceinline__ int gscan(int v, int k)
{
    int x = dpp_pin(__builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false));   // row_shr:1
    v += k >= 1 ? x : 0;
    x = dpp_pin(__builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false));       // row_shr:2
    v += k >= 2 ? x : 0;
    if constexpr (G >= 8) {
        x = dpp_pin(__builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false));
        v += k >= 4 ? x : 0;
    }
    if constexpr (G >= 16) {
        x = dpp_pin(__builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false));
        v += k >= 8 ? x : 0;
    }
    return v;
}

// f(integral_constant<int, J>) for J = 0 .. N-1, unrolled at compile time
template <typename F, int... I>
__device__ __forceinline__ void unroll_seq(F &&f, std::integer_sequence<int, I...>)
{
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void unroll(F &&f)
{
    unroll_seq(f, std::make_integer_sequence<int, N>{});
}

// number of zero bytes of x (exact: no borrow between bytes)
__device__ __forceinline__ int zero_bytes(uint32_t x)
{
    const uint32_t t = ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x | 0x7f7f7f7fu);
    return __popc(t);
}

// Observation stores (the step's bulk output, 2/3 of its bytes) as
// non-temporal stores: streamed past the caches, so they do not evict the env
// state the next step's k_logic reads (cfg3 0.0929 -> 0.0908 ms, round 3).
// (Round 5: write-back stores measured slower in the step -- cfg3 0.0846 ->
// 0.0887 ms, cfg5 0.1019 -> 0.1184 -- although a lone store stream reaches
// 5.3 TB/s with them against 4.5 TB/s non-temporal, scripts/microbench/storebw.hip.)
template <typename T>
__device__ __forceinline__ void obs_store(T *p, const T &v)
{
    __builtin_nontemporal_store(v, p);
}
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));

// The table encode's observation stores as raw buffer stores on the env's
// observation (a wave-uniform descriptor: no 64-bit address per store) with an
// explicit cache policy, SNAKE_OBS_POLICY: 0 non-temporal (as obs_store), 16
// sc1 (write-through), 17 sc0 sc1. Round 6, same box, ms per step: write-through
// would leave no dirty lines for the kernel-end writeback but measured slower
// (cfg3 0.0821 -> 0.0985, cfg5 0.0812 -> 0.0982, cfg4 0.0546 -> 0.0570; cfg3s8
// 0.0390 -> 0.0387); the buffer form itself, non-temporal, is kept: cfg4
// 0.0556 -> 0.0549, cfg3 and the driver window equal (profiles/r06_ab_obs_policy.txt).
#ifndef SNAKE_OBS_POLICY
#define SNAKE_OBS_POLICY 0
#endif
__device__ __forceinline__ void obs_store_rs(__amdgpu_buffer_rsrc_t rs, int byte_off, v4u v)
{
    if constexpr (SNAKE_OBS_POLICY == 0) __builtin_amdgcn_raw_buffer_store_b128(v, rs, byte_off, 0, 2);   // (nt)
    else __builtin_amdgcn_raw_buffer_store_b128(v, rs, byte_off, 0, SNAKE_OBS_POLICY);
}

// (Round 6: storing the two 128-byte lines an env's observation shares with
// its neighbours write-back, the rest non-temporal, measured slower in the step
// -- the per-store edge test in the encodes' store loops cost more than the
// merged lines saved: cfg3 0.0830 -> 0.0848 ms, driver window 0.0866 -> 0.0915,
// cfg5 k_post_lean 57 -> 75 us; profiles/r06_ab_edge_removed.txt.)

// k_logic with one frame writes back only the 16-byte chunks of the frame the
// step changed (0: the whole frame, as before round 6)
#ifndef SNAKE_LOGIC_DIRTY
#define SNAKE_LOGIC_DIRTY 1
#endif
#ifndef SNAKE_LOGIC_COMMIT_GROUP
#define SNAKE_LOGIC_COMMIT_GROUP 1
#endif

constexpr int kRespawnT = 4;   // raws per lane prefetched by the fast fruit respawn

__device__ __forceinline__ uint32_t gen_mask(uint32_t m)
{
    m |= m >> 1; m |= m >> 2; m |= m >> 4; m |= m >> 8; m |= m >> 16;
    return m;
}

// ---------------------------------------------------------------- MT19937
// numpy legacy RandomState stream (mt19937_seed / mt19937_gen / tempering).
// The 624-word key lives in registers: lane l holds words 64t + l, t = 0..9.
struct WaveMT {
    uint32_t w[10];
    int pos;
};

__device__ __forceinline__ uint32_t temper(uint32_t y)
{
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

// m.w[t] for a wave-uniform runtime t. Masked ORs, not selects: InstCombine turns
// a select of two loads into a load through a selected pointer, which would
// demote the whole register array to scratch.
__device__ __forceinline__ uint32_t word_at(const WaveMT &m, int t)
{
    uint32_t v = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) v |= m.w[i] & (0u - (uint32_t)(t == i));
    return v;
}

__device__ __forceinline__ void mt_load(WaveMT &m, const uint32_t *g, int pos, int lane)
{
#pragma unroll
    for (int t = 0; t < 10; t++) {
        const int e = 64 * t + lane;
        m.w[t] = (e < kMtN) ? g[e] : 0u;
    }
    m.pos = pos;
}

__device__ __forceinline__ void mt_store(const WaveMT &m, uint32_t *g, int lane)
{
#pragma unroll
    for (int t = 0; t < 10; t++) {
        const int e = 64 * t + lane;
        if (e < kMtN) g[e] = m.w[t];
    }
}

// mt19937_gen, wave-parallel. new[i] = X ^ (y >> 1) ^ mag(y), y = old[i]|old[i+1]
// (upper/lower bits), X = old[i+397] for i < 227 and new[i-227] after; the last
// word mixes new[0]. Every element's inputs sit at a fixed lane offset (13 for
// i+397, 29 for i-227) of an earlier register, so the twist is 10 register
// steps in four dependency levels (registers {0-2}, {3-5}, {6-8}, {9}); the
// cross-lane reads of a level are issued together.
__device__ __forceinline__ uint32_t mt_mix(uint32_t cur, uint32_t nxt, uint32_t x)
{
    const uint32_t y = (cur & 0x80000000u) | (nxt & 0x7fffffffu);
    return x ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

__device__ void mt_twist(WaveMT &m, int lane)
{
    const int l1 = (lane + 1) & 63, l13 = (lane + 13) & 63, l29 = (lane + 29) & 63;
    const bool wrap13 = lane + 13 >= 64, wrap29 = lane + 29 >= 64;
    uint32_t o1[10], xo[4], nw[10];
    // level 0: everything that reads old words only
#pragma unroll
    for (int t = 0; t < 10; t++) {
        const uint32_t same = __shfl(m.w[t], l1);
        const uint32_t nxt = __builtin_amdgcn_readlane(m.w[t < 9 ? t + 1 : 9], 0);
        o1[t] = (lane == 63) ? nxt : same;
    }
#pragma unroll
    for (int t = 0; t < 4; t++) {
        const uint32_t a = __shfl(m.w[t + 6], l13);
        const uint32_t b = __shfl(m.w[t + 7 <= 9 ? t + 7 : 9], l13);
        xo[t] = wrap13 ? b : a;
    }
#pragma unroll
    for (int t = 0; t < 3; t++) nw[t] = mt_mix(m.w[t], o1[t], xo[t]);
    // levels 1..3: X = new[i-227] = register t-4 (or t-3 past the lane wrap)
#pragma unroll
    for (int lv = 1; lv <= 3; lv++) {
        const int t0 = 3 * lv, t1 = (lv == 3) ? 10 : 3 * lv + 3;
        uint32_t xn[3];
#pragma unroll
        for (int t = t0; t < t1; t++) {
            const uint32_t a = __shfl(nw[t >= 4 ? t - 4 : 0], l29);
            const uint32_t b = __shfl(nw[t - 3], l29);
            xn[t - t0] = wrap29 ? b : a;
        }
        uint32_t n0 = 0, n396 = 0;
        if (lv == 3) {
            n0 = __builtin_amdgcn_readlane(nw[0], 0);
            n396 = __builtin_amdgcn_readlane(nw[6], 12);
        }
#pragma unroll
        for (int t = t0; t < t1; t++) {
            const int e = 64 * t + lane;
            uint32_t x = xn[t - t0], nx = o1[t];
            if (t == 3) x = (e < 227) ? xo[3] : x;
            if (t == 9 && e == kMtN - 1) { nx = n0; x = n396; }
            const uint32_t v = mt_mix(m.w[t], nx, x);
            nw[t] = (e < kMtN) ? v : 0u;
        }
    }
#pragma unroll
    for (int t = 0; t < 10; t++) m.w[t] = nw[t];
    m.pos -= kMtN;   // a pending twist: position 624 + j is word j of the new key
}

// One masked bounded draw: first raw r (in stream order) with (r & mask) <= rng.
// randint's masked rejection (grid_util.py:130); the caller handles rng == 0.
__device__ uint32_t mt_draw(WaveMT &m, uint32_t mask, uint32_t rng, int lane)
{
    for (;;) {
        if (m.pos >= kMtN) mt_twist(m, lane);
        const int t = m.pos >> 6, l0 = m.pos & 63;
        const uint32_t v = temper(word_at(m, t)) & mask;
        const int e = (t << 6) + lane;
        const unsigned long long b = __ballot(lane >= l0 && e < kMtN && v <= rng);
        if (b) {
            const int f = __ffsll((long long)b) - 1;
            m.pos = (t << 6) + f + 1;
            return (uint32_t)bcast((int)v, f);
        }
        m.pos = min((t + 1) << 6, kMtN);
    }
}

// set bits of x below this lane, + add
__device__ __forceinline__ int mbcnt64(unsigned long long x, int add = 0)
{
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(x >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)x, (uint32_t)add));
}

// this lane's bit of a wave mask, as a lane predicate (v_cndmask on the SGPR pair)
__device__ __forceinline__ bool inv_ballot(unsigned long long m) { return __builtin_amdgcn_inverse_ballot_w64(m); }

// permutation(n) = shuffle(arange(n)) draws j_i = random_interval(i) for
// i = n-1 .. 1 (snake_env.py:581). Only arr[0..S) is ever used, so instead of the
// draws themselves the pass records, for the backward trace (perm_trace):
//   jsmall[i] = j_i for i < S, and link[x] = min{ i >= S : j_i = x < i }.
// A round covers the unread raw words of one aligned register pair (2q, 2q+1):
// lane l holds the words at stream offsets p = l - l0 (first register) and
// 64 - l0 + l (second). A word is accepted iff (w & mask) <= i - A_p, A_p = the
// accepts before it. The accept set is found by bound refinement: with acc (sure
// accepts) and pos (possible accepts) every lane knows L = |acc before it| <= A_p
// <= U = |pos before it|, and re-deciding every lane against both bounds fixes at
// least the first undecided lane per pass (typically 1-2 passes). Words past the
// accept that takes i below the current power-of-two bracket were judged with
// the wrong mask: the round ends right after that accept.
template <typename NP>
__device__ __forceinline__ void perm_record(int ii, int w, int S, NP *link, lu16 *jsmall)
{
    if (ii < S) jsmall[ii] = (uint16_t)w;
    else if (w != ii) link_min(link + w, (uint32_t)ii);
}

// One draw round over the unread words of the register pair (tw0, tw1) at key
// offset base (see mt_perm_draws). Bound refinement from the possible set:
// c = {w <= i} is a superset of the accepts, a = {w + |c before| <= i} a
// subset; a == c settles the round (most rounds, in one pass: only a word
// within |c before p| - A_p of its threshold stays open), else the bounds
// alternate until they meet. The accept set's prefix counts b are the draw
// indices' offsets, and the draw record is written through a per-lane dummy
// slot instead of exec masking: under the step's load the worker waves are
// issue-bound, so instructions (SALU and branches included) are the cost.
// population count of a wave mask on the vector ALU (`ones` is an opaque
// all-ones VGPR): the scalar count of a mask a vector compare just wrote costs a
// vector-to-scalar hand-off and a move back in the round's dependency chain
__device__ __forceinline__ int vpopc(unsigned long long x, uint32_t ones)
{
    return __builtin_popcount((uint32_t)x & ones) + __builtin_popcount((uint32_t)(x >> 32) & ones);
}

// Returns true when the round ended at a bracket cut inside the pair with
// draws left: the next round reads the same register pair.
template <typename NP>
__device__ __forceinline__ bool draw_round(uint32_t tw0, uint32_t tw1, int base, WaveMT &m, int &i,
                                           uint32_t &mask, int &lo, int S, NP *link, NP *dummy,
                                           lu16 *jsmall, uint32_t ones, int lane)
{
    constexpr int kBig = 0x3fffffff;   // never accepted; w + b cannot overflow
    const int l0 = m.pos - base;
    const int p0 = lane - l0;   // stream offset of this lane's first word (second: + 64)
    const int w0 = p0 >= 0 ? (int)(tw0 & mask) : kBig;
    const int w1 = (p0 >= -64 && base + 64 + lane < kMtN) ? (int)(tw1 & mask) : kBig;
    unsigned long long c0 = __ballot(w0 <= i), c1 = __ballot(w1 <= i);
    int b0 = mbcnt64(c0), b1 = mbcnt64(c1, vpopc(c0, ones));
    unsigned long long a0 = __ballot(w0 + b0 <= i), a1 = __ballot(w1 + b1 <= i);
    // (the empty asm keeps each test on the OR of both halves: folded into two
    // 64-bit compares it costs two selects and an AND per test)
    unsigned long long und = (a0 ^ c0) | (a1 ^ c1);
    __asm__ volatile("" : "+s"(und));
    if (__builtin_expect(und != 0ull, 0)) {
        for (int pass = 0; pass < 128; pass++) {
            b0 = mbcnt64(a0);
            b1 = mbcnt64(a1, __popcll(a0));
            c0 = __ballot(w0 + b0 <= i);
            c1 = __ballot(w1 + b1 <= i);
            und = (a0 ^ c0) | (a1 ^ c1);
            __asm__ volatile("" : "+s"(und));
            if (und == 0ull) break;
            b0 = mbcnt64(c0);
            b1 = mbcnt64(c1, __popcll(c0));
            a0 = __ballot(w0 + b0 <= i);
            a1 = __ballot(w1 + b1 <= i);
            und = (a0 ^ c0) | (a1 ^ c1);
            __asm__ volatile("" : "+s"(und));
            if (und == 0ull) break;
        }
    }
    // a == c: b0, b1 = the accepts before each word
    const int A0 = __popcll(a0);
    int A = A0 + __popcll(a1);
    int end = min(128, kMtN - base);
    const int k = i - lo + 1;  // accepts left in this bracket
    bool cut = false;
    if (__builtin_expect(A >= k, 0)) {
        cut = true;
        if (A0 >= k) {
            const int b = __ffsll((long long)__ballot(inv_ballot(a0) && b0 == k - 1)) - 1;
            a0 &= (2ull << b) - 1ull;
            a1 = 0;
            end = b + 1;
        } else {
            const int b = __ffsll((long long)__ballot(inv_ballot(a1) && b1 == k - 1)) - 1;
            a1 &= (2ull << b) - 1ull;
            end = 64 + b + 1;
        }
        A = k;
    }
    const int ii0 = i - b0, ii1 = i - b1;
    if constexpr (std::is_same<NP, lu16>::value) {
        // LDS draw record: j_i at index i (one writer per index), the rest to
        // the lane's dummy slot
        *(inv_ballot(a0) ? link + ii0 : dummy) = (uint16_t)w0;
        *(inv_ballot(a1) ? link + ii1 : dummy) = (uint16_t)w1;
    } else if (__builtin_expect(i - A + 1 < S, 0)) {   // the last rounds: some indices < S
        if (inv_ballot(a0)) perm_record(ii0, w0, S, link, jsmall);
        if (inv_ballot(a1)) perm_record(ii1, w1, S, link, jsmall);
    } else {
        // every index of the round >= S: unconditional min, misses to the dummy
        link_min((inv_ballot(a0) && w0 != ii0) ? link + w0 : dummy, (uint32_t)ii0);
        link_min((inv_ballot(a1) && w1 != ii1) ? link + w1 : dummy, (uint32_t)ii1);
    }
    m.pos = base + end;
    i -= A;
    // the bracket of the new i, branch-free (i < 1 ends the draws anyway)
    mask = i > 0 ? (0xffffffffu >> __builtin_clz((uint32_t)i)) : 0u;
    lo = (int)(mask >> 1) + 1;
    return cut && i >= 1 && end < 128 && m.pos < kMtN;
}


template <typename NP>
__device__ void mt_perm_draws(WaveMT &m, int n, int S, NP *link, int link_n, lu16 *jsmall, int lane)
{
    int i = n - 1;
    if (i < 1) return;
    uint32_t mask = gen_mask((uint32_t)i);
    int lo = (int)(mask >> 1) + 1;
    // the tempered key stays in registers: the rounds never read LDS, so nothing
    // waits for the link-table atomics until the draws are done. The rounds of a
    // key block run pair by pair, unrolled: each pair's words are fixed registers.
    uint32_t tk[10];
#pragma unroll
    for (int t = 0; t < 10; t++) tk[t] = temper(m.w[t]);
    NP *dummy = link + link_n + lane;   // lanes with nothing to record hit their own dummy
    uint32_t ones;
    __asm__ volatile("v_mov_b32 %0, -1" : "=v"(ones));
    // every round advances the stream; the cap only guarantees that a broken
    // invariant ends the wave instead of hanging the GPU
    for (int guard = 0; i >= 1 && guard < (1 << 20); guard++) {
        if (m.pos >= kMtN) {
            mt_twist(m, lane);
#pragma unroll
            for (int t = 0; t < 10; t++) tk[t] = temper(m.w[t]);
        }
#pragma unroll
        for (int q = 0; q < 5; q++) {
            // a round normally consumes the rest of the pair; only a bracket cut
            // inside it repeats the pair
            if (i >= 1 && m.pos < kMtN && (m.pos >> 7) == q) {
                bool again;
                do {
                    again = draw_round(tk[2 * q], tk[2 * q + 1], q << 7, m, i, mask, lo, S, link, dummy, jsmall,
                                       ones, lane);
                } while (__builtin_expect(again, 0));
            }
        }
    }
}

// Final arr[k] of the Fisher-Yates pass for k < S from the LDS draw record
// (jarr[i] = j_i): replay the swaps i < S on lane k's position k, then scan
// i = S .. n-1 in order, 256 at a time: a tracked position x moves to i exactly
// when j_i == x (the swap brings arr[i] there; x < i always). Every tracked
// position is tested against a chunk with one ballot; a hit re-tests the rest
// of the chunk from the new position.
template <int MS>
__device__ void perm_trace_j(int S, int n, const lu16 *jarr, int (&q)[MS], int lane)
{
    int x = lane;
    for (int i = 1; i < S; i++) {
        const int j = jarr[i];
        x = (x == i) ? j : (x == j ? i : x);
    }
    // tracked positions, and as packed 16-bit pairs for the match test
    // (positions and record entries are < 65 535; untracked slots and the
    // padding past n are 0xffff: a padding match only sends the last chunk down
    // the exact per-position path)
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    int xk[MS];
    u16x2 xp[MS / 2];
#pragma unroll
    for (int k = 0; k < MS; k++) xk[k] = bcast(x, k);
    auto pack = [&]() {
#pragma unroll
        for (int p2 = 0; p2 < MS / 2; p2++) {
            xp[p2].x = (unsigned short)(2 * p2 < S ? xk[2 * p2] : 0xffff);
            xp[p2].y = (unsigned short)(2 * p2 + 1 < S ? xk[2 * p2 + 1] : 0xffff);
        }
    };
    pack();
    for (int base = S; base < n; base += 4 * kWave) {
        int jv[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int i = base + u * kWave + lane;
            jv[u] = (int)jarr[min(i, n - 1)];
            jv[u] = i < n ? jv[u] : 0xffff;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            // one ballot against every tracked position (a move is rare: ~ln n
            // per position over the whole scan); the per-position chase only
            // when some lane matched
            // (packed 16-bit differences to two tracked positions per vector
            // instruction, their minimum; zero = a match: one vector-to-scalar
            // hand-off per block)
            u16x2 jj;
            jj.x = (unsigned short)jv[u];
            jj.y = (unsigned short)jv[u];
            u16x2 dm = jj - xp[0];
#pragma unroll
            for (int p2 = 1; p2 < MS / 2; p2++) dm = __builtin_elementwise_min(dm, jj - xp[p2]);
            const bool hit = min(dm.x, dm.y) == 0;
            if (__builtin_expect(__ballot(hit) != 0ull, 0)) {
#pragma unroll
                for (int k = 0; k < MS; k++) {
                    if (k < S) {
                        unsigned long long m = __ballot(jv[u] == xk[k]);
                        while (m) {
                            const int l = __ffsll((long long)m) - 1;
                            xk[k] = base + u * kWave + l;
                            m = __ballot(jv[u] == xk[k]);
                        }
                    }
                }
                pack();
            }
        }
    }
#pragma unroll
    for (int k = 0; k < MS; k++) q[k] = xk[k];
}

// Final arr[k] of the Fisher-Yates pass for k < S, lane k: walk position k
// backwards through the swaps (i ascending). The swaps i < S only move positions
// < S (j_i <= i): replay them from jsmall. After that the tracked position q < S
// <= i is only moved by a swap with j_i = q, to position i; from position x the
// next move is the first later swap with j = x: link[x]. Chains are ~ln(n) long.
template <int MS, typename NP>
__device__ void perm_trace(int S, const NP *link, const lu16 *jsmall, int (&q)[MS], int lane)
{
    int x = lane;
    for (int i = 1; i < S; i++) {
        const int j = jsmall[i];
        x = (x == i) ? j : (x == j ? i : x);
    }
    if (lane < S) {
        for (;;) {
            const uint32_t y = link_get(link + x);
            if (y == kNoLink) break;
            x = (int)y;
        }
    }
#pragma unroll
    for (int k = 0; k < MS; k++) q[k] = bcast(x, k);
}


// ------------------------------------------------------------ fruit respawn
// random_empty_coords + grid[xs, ys] = FRUIT (grid_util.py:126-133,
// snake_env.py:376-379): np.where order is row-major, draws are with
// replacement, all draws index the pre-respawn empty list.
__device__ void place_fruits(const KCfg &c, uint8_t *g, WaveMT &m, int k, uint16_t *fbuf, int lane)
{
    const int c0 = lane * c.cs, c1 = min(c.HW, c0 + c.cs);
    int cnt = 0;
    for (int x = c0; x < c1; x++) cnt += (g[x] == C_EMPTY);
    const int incl = wave_scan(cnt, lane), excl = incl - cnt;
    const int E = bcast(incl, 63);
    if (E == 0) return;  // no empty cell: no draw (random_empty_coords returns None)
    const uint32_t rng = (uint32_t)(E - 1), mask = gen_mask(rng);
    for (int d = 0; d < k; d++) {
        const uint32_t v = rng == 0 ? 0u : mt_draw(m, mask, rng, lane);
        if ((int)v >= excl && (int)v < incl) {
            int need = (int)v - excl;
            for (int x = c0; x < c1; x++) {
                if (g[x] == C_EMPTY) {
                    if (need == 0) { fbuf[d] = (uint16_t)x; break; }
                    need--;
                }
            }
        }
    }
    wave_sync();
    for (int d = lane; d < k; d += kWave) g[fbuf[d]] = C_FRUIT;
    wave_sync();
}


// The reset's fruits (SnakeEnv.reset :147-148 -> random_empty_coords,
// grid_util.py:126-133) on the freshly painted board: its empty cells are the
// interior minus the S*L disjoint snake cells, so no grid scan is needed.
// Draws: randint(0, E, size=k), one mt_draw each (all index the same empty
// list: placing a fruit does not change E).
// Cells: the v-th empty cell in np.where's row-major order has interior index
// y = the least fixed point of y = v + #{snake cells with interior index <= y}
// (iterated from v: a snake cell is never a least fixed point). `cell` = lane's
// snake cell (lanes < S*L).
__device__ void place_fruits_fresh(const KCfg &c, uint8_t *g, WaveMT &m, int k, int cell, int lane)
{
    const int Wi = c.W - 2, SL = c.S * c.L;
    const uint32_t E = (uint32_t)((c.H - 2) * Wi - SL), rng = E - 1, mask = gen_mask(rng);
    const int hr = (int)__umulhi((uint32_t)cell, c.mag_W);
    const int yi = lane < SL ? (hr - 1) * Wi + (cell - hr * c.W - 1) : INT_MAX;
    for (int d = 0; d < k; d++) {
        // randint(0, E) (rng == 0: no raw consumed), the same mt_draw as the step's respawn
        const int v = rng == 0 ? 0 : (int)mt_draw(m, mask, rng, lane);
        int y = v;
        for (int it = 0; it <= SL; it++) {
            const int y1 = v + __popcll(__ballot(yi <= y));
            if (y1 == y) break;
            y = y1;
        }
        const int r = y / Wi;
        if (lane == 0) g[(r + 1) * c.W + (y - r * Wi) + 1] = C_FRUIT;
    }
    wave_sync();
}

// ------------------------------------------------------------------ encode
// _encode (snake_env.py:474-519) + frame stack (:444-472): for snake k the 8
// channels [wall, fruit, other head/body/tail, own head/body/tail]; with a vision
// range the (2vr+1)^2 window is centred on the own-HEAD cell (argmax of the own
// head plane: the snake's head while alive, (0,0) once dead) and zero outside
// the grid. org[f*16+k] = crop origin of snake k in frame f, packed
// ((r0 + 256) << 16) | (c0 + 256).
__device__ __forceinline__ unsigned long long onehot(int v, int k)
{
    const int id = div10(v);
    const int code = v - 10 * id;                   // 3 HEAD, 4 BODY, 5 TAIL
    const int ch = (v < 3) ? v - 1 : ((id == k) ? code + 2 : code - 1);
    return v == C_EMPTY ? 0ull : (1ull << (8 * ch));
}

__device__ __forceinline__ unsigned long long unit_bits(const KCfg &c, const uint8_t *frames,
                                                       const int *org, int k, int i, int j, int s)
{
    const int p = org[s * kMaxSnakes + k];
    const int r = (p >> 16) - 256 + i, cc = (p & 0xffff) - 256 + j;
    if ((unsigned)r >= (unsigned)c.H || (unsigned)cc >= (unsigned)c.W) return 0ull;
    return onehot(frames[s * c.grid_stride + r * c.W + cc], k);
}

// obs layout (S, oh, ow, 8*fs): unit u = ((k*oh + i)*ow + j)*fs + f is 8 bytes;
// frame f (oldest first) is ring slot (slot0 + f) % fs of the LDS ring.
// Lane l writes units 2l, 2l+1 (16 bytes) then strides by 128 units; the
// (k,i,j,f) digits advance by carries, no division in the loop.
__device__ void encode(const KCfg &c, const uint8_t *frames, const int *org, int slot0,
                       uint8_t *obs_env, int lane)
{
    const int U = c.units, pairs = (U + 1) >> 1, fs = c.fs;
    int u = 2 * lane;
    int f = u % fs, rest = u / fs;
    int j = rest % c.ow;
    rest /= c.ow;
    int i = rest % c.oh;
    int k = rest / c.oh;
    const bool wide = (U & 1) == 0;
    for (int p = lane; p < pairs; p += kWave) {
        int s = slot0 + f;
        s -= (s >= fs) ? fs : 0;
        const unsigned long long a = unit_bits(c, frames, org, k, i, j, s);
        int f2 = f + 1, j2 = j, i2 = i, k2 = k;
        if (f2 == fs) {
            f2 = 0;
            if (++j2 == c.ow) { j2 = 0; if (++i2 == c.oh) { i2 = 0; k2++; } }
        }
        int s2 = slot0 + f2;
        s2 -= (s2 >= fs) ? fs : 0;
        const bool has_b = 2 * p + 1 < U;
        const unsigned long long b = has_b ? unit_bits(c, frames, org, k2, i2, j2, s2) : 0ull;
        if (wide) {
            uint4 v;
            v.x = (uint32_t)a; v.y = (uint32_t)(a >> 32);
            v.z = (uint32_t)b; v.w = (uint32_t)(b >> 32);
            obs_store(reinterpret_cast<v4u *>(obs_env + 16 * (int64_t)p), (v4u){v.x, v.y, v.z, v.w});
        } else {
            obs_store(reinterpret_cast<unsigned long long *>(obs_env + 16 * (int64_t)p), a);
            if (has_b) obs_store(reinterpret_cast<unsigned long long *>(obs_env + 16 * (int64_t)p + 8), b);
        }
        f += c.adv_f;
        if (f >= fs) { f -= fs; j++; }
        j += c.adv_j;
        if (j >= c.ow) { j -= c.ow; i++; }
        i += c.adv_i;
        if (i >= c.oh) { i -= c.oh; k++; }
        k += c.adv_k;
    }
}

// Lean encode (k_encode): the observation straight from a zero-bordered copy
// of the env's frames in LDS (pf: frame s's grid cell (r, c) at s*pframe +
// (r + vr)*pw + c + lp, zero around it), so a crop window never needs a bounds
// test; base[s*16 + k] = the LDS offset of snake k's window origin in frame s
// (0 for the full map). Lane = one 16-byte output chunk = two consecutive
// units (8 obs bytes each: one cell of one frame): per unit one LDS byte read
// and its one-hot channel (_encode :481-492), no LDS staging of the output, no
// divergent branch.
template <int T = kWave>
__device__ void encode_lean(const KCfg &c, const uint8_t *pf, const int *base, int slot0, uint8_t *obs_env,
                            int lane)
{
    const int pairs = c.units >> 1;
    for (int p = lane; p < pairs; p += T) {
        const uint32_t u = 2u * (uint32_t)p;
        int kk = (int)__umulhi(u, c.mag_ups);
        const int r0 = (int)u - kk * c.ups;
        int ii = (int)__umulhi((uint32_t)r0, c.mag_rowl);
        const int r1 = r0 - ii * c.rowl;
        int jj = fdiv((uint32_t)r1, c.mag_fs, c.fs);
        int ff = r1 - jj * c.fs;
        uint32_t w[4];
#pragma unroll
        for (int h = 0; h < 2; h++) {
            int s = slot0 + ff;
            s -= (s >= c.fs) ? c.fs : 0;
            const int v = pf[s * c.pframe + base[s * kMaxSnakes + kk] + ii * c.pw + jj];
            const int id = div10(v), code = v - 10 * id;
            const int ch = (v < 3) ? v - 1 : ((id == kk) ? code + 2 : code - 1);
            const uint32_t bit = (v != 0) ? (1u << (8 * (ch & 3))) : 0u;
            w[2 * h] = ch < 4 ? bit : 0u;
            w[2 * h + 1] = ch < 4 ? 0u : bit;
            if (h == 0) {   // the next unit: frame, then column, row, snake digits carry
                ff++;
                const bool cf = ff == c.fs;
                ff = cf ? 0 : ff;
                jj += cf;
                const bool cj = jj == c.ow;
                jj = cj ? 0 : jj;
                ii += cj;
                const bool ci = ii == c.oh;
                ii = ci ? 0 : ii;
                kk += ci;
            }
        }
        obs_store(reinterpret_cast<v4u *>(obs_env) + p, (v4u){w[0], w[1], w[2], w[3]});
    }
}

// env e's frames into the zero-bordered LDS image of encode_lean (the border
// was zeroed by the caller and is never written) and its window origins.
__device__ void stage_lean(const KCfg &c, const snake_state &st, int64_t e, uint8_t *pf, int *base, int lane)
{
    const uint8_t *ring = st.grid + e * c.ring_bytes;
    const int tp = c.vr;
    if ((c.W & 3) == 0) {
        const int wpr = c.W >> 2, nw = c.H * wpr;
        const uint32_t *r32 = reinterpret_cast<const uint32_t *>(ring);
        uint32_t *p32 = reinterpret_cast<uint32_t *>(pf);
        for (int s = 0; s < c.fs; s++)
            for (int x = lane; x < nw; x += kWave) {
                const int r = fdiv((uint32_t)x, c.mag_wpr, wpr), c4 = x - r * wpr;
                p32[(s * c.pframe + (r + tp) * c.pw + c.lp) / 4 + c4] = r32[s * (c.grid_stride >> 2) + x];
            }
    } else {
        for (int s = 0; s < c.fs; s++)
            for (int x = lane; x < c.HW; x += kWave) {
                const int r = (int)__umulhi((uint32_t)x, c.mag_W), cc = x - r * c.W;
                pf[s * c.pframe + (r + tp) * c.pw + c.lp + cc] = ring[s * c.grid_stride + x];
            }
    }
    const int fsS = c.fs * c.S;
    if (lane < fsS) {
        const int x = lane / c.S, k = lane - x * c.S;
        const int p = st.ctr[e * fsS + lane];
        base[x * kMaxSnakes + k] = c.vr ? (p >> 8) * c.pw + (p & 255) + c.lp - c.vr : 0;
    }
}

template <int T = kWave>
__device__ __forceinline__ void zero_lean(const KCfg &c, uint8_t *pf, int lane)
{
    for (int q = lane; q < (c.fs * c.pframe) >> 4; q += T) reinterpret_cast<uint4 *>(pf)[q] = make_uint4(0, 0, 0, 0);
}

// Row-wise encode: lane = one (snake, frame, window row); the row's cells are
// scattered as single bytes into a zeroed LDS image of a group of whole snakes'
// observations, which is then copied out with 16-byte stores. Per cell: one
// frame byte read, the channel, one byte write (empty cells write nothing).
__device__ void encode_rows(const KCfg &c, const uint8_t *frames, const int *org, int slot0,
                            uint8_t *obs_env, uint8_t *stage, int lane)
{
    const int fs = c.fs, ow = c.ow, oh = c.oh, S = c.S, cellb = 8 * fs, W = c.W;
    const int P = oh * ow * cellb;
    const int fsoh = fs * oh;
    const bool wide = (c.units & 1) == 0;
    for (int k0 = 0; k0 < S; k0 += c.enc_group) {
        const int gs = min(c.enc_group, S - k0), bytes = gs * P;
        for (int q = lane; q < (bytes + 15) >> 4; q += kWave)
            reinterpret_cast<uint4 *>(stage)[q] = make_uint4(0, 0, 0, 0);
        wave_sync();
        for (int rr = lane; rr < gs * fsoh; rr += kWave) {
            const int kk = (int)__umulhi((uint32_t)rr, c.mag_fsoh), rem = rr - kk * fsoh;
            const int f = (int)__umulhi((uint32_t)rem, c.mag_oh), i = rem - f * oh;
            const int k = k0 + kk;
            int s = slot0 + f;
            s -= (s >= fs) ? fs : 0;
            const int p = org[s * kMaxSnakes + k];
            const int r = (p >> 16) - 256 + i, c0 = (p & 0xffff) - 256;
            if ((unsigned)r >= (unsigned)c.H) continue;
            const uint8_t *row = frames + s * c.grid_stride + r * W;
            uint8_t *dst = stage + kk * P + i * ow * cellb + f * 8;
            for (int j = 0; j < ow; j++) {
                const int cc = c0 + j;
                const int v = ((unsigned)cc < (unsigned)W) ? row[cc] : 0;
                const int id = div10(v), code = v - 10 * id;
                const int ch = (v < 3) ? v - 1 : code - 1 + ((id == k) ? 3 : 0);
                if (v != 0) dst[j * cellb + ch] = 1;
            }
        }
        wave_sync();
        uint8_t *out = obs_env + (int64_t)k0 * P;
        if (wide) {
            for (int q = lane; q < bytes >> 4; q += kWave)
                obs_store(reinterpret_cast<v4u *>(out) + q, reinterpret_cast<const v4u *>(stage)[q]);
        } else {
            for (int q = lane; q < bytes >> 3; q += kWave)
                obs_store(reinterpret_cast<v2u *>(out) + q, reinterpret_cast<const v2u *>(stage)[q]);
        }
        wave_sync();
    }
}

__device__ __forceinline__ void encode_obs(const KCfg &c, const uint8_t *frames, const int *org, int slot0,
                                           uint8_t *obs_env, uint8_t *lds, int lane)
{
    if (c.enc_group > 0) encode_rows(c, frames, org, slot0, obs_env, lds + c.lds_stage, lane);
    else encode(c, frames, org, slot0, obs_env, lane);
}

__device__ __forceinline__ int pack_origin(const KCfg &c, int r, int cc)
{
    return c.vr ? (((r - c.vr + 256) << 16) | (cc - c.vr + 256)) : ((256 << 16) | 256);
}

__device__ __forceinline__ int dir_of_diff(int diff, int W)
{
    return diff == -W ? 0 : (diff == 1 ? 1 : (diff == W ? 2 : 3));
}

// ------------------------------------------------------------------- reset
// One iteration of _generate_snakes' retry loop (:576-589): S spawn poses =
// permutation(n_cand)[:S] drawn from the wave's MT, lane (sk, si) = cell si of
// pose sk (-1 past S*L), q = the pose indices; true when the poses are disjoint
// (_clear_overlap :568-574).
template <int MS, int JL>
__device__ bool spawn_attempt(const KCfg &c, const snake_state &st, WaveMT &mt, uint8_t *lds, int slot,
                              int (&q)[MS], int &cell, int lane)
{
    const int S = c.S, L = c.L, SL = S * L;
    const int sk = lane / L, si = lane - sk * L;
    if constexpr (JL == 2) {
        {
            // small batches: the u32 link table in LDS (ds_min, no scan: the
            // trace is a short pointer chase)
            lu32 *link = (lu32 *)(lds + c.lds_link);
            lu16 *jsmall = (lu16 *)(lds + c.lds_fruit);   // the fruit buffer is free until place_fruits
            for (int x = 4 * lane; x < c.link_stride - kWave; x += 4 * kWave) *(lu4 *)(link + x) = (v4u32)kNoLink;
            wave_sync();
            mt_perm_draws(mt, c.n_cand, S, link, c.n_cand, jsmall, lane);
            wave_sync();
            perm_trace<MS>(S, link, jsmall, q, lane);
        }
    } else if constexpr (JL == 1) {
        {
            // the u16 draw record in LDS: every index 1..n-1 is written, nothing to clear
            lu16 *jarr = (lu16 *)(lds + c.lds_link);
            mt_perm_draws(mt, c.n_cand, S, jarr, c.n_cand, jarr, lane);
            wave_sync();
            perm_trace_j<MS>(S, c.n_cand, jarr, q, lane);
        }
    } else {
        // large boards: the link table in this worker's global scratch
        gu32 *link = (gu32 *)(st.jscratch + (int64_t)slot * c.link_stride);
        lu16 *jsmall = (lu16 *)(lds + c.lds_fruit);   // the fruit buffer is free until place_fruits
        for (int x = 4 * lane; x < c.link_stride - kWave; x += 4 * kWave)
            *(gu4 *)(link + x) = (v4u32)kNoLink;
        // (the table is this wave's alone: its own stores and atomics drained
        // and made visible, no workgroup barrier -- k_post_lean runs four
        // independent workers per workgroup)
        link_sync();
        mt_perm_draws(mt, c.n_cand, S, link, c.n_cand, jsmall, lane);
        link_sync();   // the link table, written by every lane
        perm_trace<MS>(S, link, jsmall, q, lane);
    }
    int pk = 0;
#pragma unroll
    for (int k = 0; k < MS; k++) pk = (sk == k) ? q[k] : pk;
    cell = (lane < SL) ? (int)st.cand[(int64_t)pk * L + si] : -1;
    bool dup = false;
    for (int x = 0; x < SL; x++) {
        const int cx = bcast(cell, x);
        dup |= (lane < SL && lane != x && cx == cell);
    }
    return __ballot(dup) == 0ull;
}

// Spawn-ahead status word (env word ENV_SPAWN): bits 0-1 the status, bit 2 the
// record buffer holding the record (background spawn-ahead keeps two per env,
// k_spawn), bits 3-31 the generation (bumped by every draw that voids it).
constexpr uint32_t kGenOne = 1u << kSpawnGenShift;
__device__ __forceinline__ uint32_t *spawn_rec(const KCfg &c, const snake_state &st, int64_t e, int b)
{
    return st.spawn + ((int64_t)b * c.N + e) * kSpawnStride;
}

// Hand-off of a record between concurrently running kernels (background
// spawn-ahead): write-through (sc1) stores, drained, then the status word's
// compare-and-swap; the reader takes the word with an atomic and loads the
// record with sc1 loads (MI355X_MICROARCH.md, inter-workgroup visibility).
__device__ __forceinline__ uint32_t ld_sc1(const uint32_t *p)
{
    return __hip_atomic_load((const gu32 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(uint32_t *p, uint32_t v)
{
    __hip_atomic_store((gu32 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 8-byte forms (global address space: never flat), and 16 bytes as two of them
typedef __attribute__((address_space(1))) unsigned long long gu64;
__device__ __forceinline__ unsigned long long ld_sc1_64(const void *p)
{
    return __hip_atomic_load((const gu64 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1_64(void *p, unsigned long long v)
{
    __hip_atomic_store((gu64 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1_128(void *p, uint4 v)
{
    st_sc1_64(p, (unsigned long long)v.x | ((unsigned long long)v.y << 32));
    st_sc1_64((uint8_t *)p + 8, (unsigned long long)v.z | ((unsigned long long)v.w << 32));
}
__device__ __forceinline__ uint4 ld_sc1_128(const void *p)
{
    const unsigned long long a = ld_sc1_64(p), b = ld_sc1_64((const uint8_t *)p + 8);
    return make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
}

__device__ __forceinline__ void mt_load_sc1(WaveMT &m, const uint32_t *g, int pos, int lane)
{
#pragma unroll
    for (int t = 0; t < 10; t++) {
        const int e = 64 * t + lane;
        m.w[t] = (e < kMtN) ? ld_sc1(g + e) : 0u;
    }
    m.pos = pos;
}

// The MT19937 state a reset (or an in-step spawn-ahead attempt) of env e
// starts from: the spawn-ahead record when one exists (the key and position
// after its recorded attempts), else the env's own; cellw = this lane's word
// of the record's spawn cells (lanes 2m, 2m + 1: word m). Returns the status
// word (wave-uniform; the status is its bits 0-1). The state it expects (the
// record for a reset, the env's own for an attempt, which mostly starts afresh)
// is loaded with the status word, in the same round trip; the other one only
// when the status asks for it. (Records are in buffer 0 without background
// spawn-ahead.)
__device__ __forceinline__ int load_reset_mt(const KCfg &c, const snake_state &st, int64_t e, WaveMT &mt, int lane,
                                             bool expect_record, uint32_t &cellw)
{
    const uint32_t *rec = spawn_rec(c, st, e, 0);
    const uint32_t *key = st.mt + e * kMtN;
    const int spw = st.env[e * kEnvRec + ENV_SPAWN];
    if (expect_record) {
        mt_load(mt, rec, (int)rec[kSpawnPos], lane);
        cellw = rec[kSpawnCells + (lane >> 1)];
        if ((spw & 3) == SPAWN_NONE) mt_load(mt, key, st.env[e * kEnvRec + ENV_MTPOS], lane);
    } else {
        mt_load(mt, key, st.env[e * kEnvRec + ENV_MTPOS], lane);
        cellw = 0;
        if ((spw & 3) != SPAWN_NONE) mt_load(mt, rec, (int)rec[kSpawnPos], lane);
    }
    return spw;
}

// Background spawn-ahead (KCfg.bg): an auto-reset takes env e's record with one
// atomic that bumps the generation (a k_spawn job still working on the env then
// fails its publish), and reads the record it found with sc1 loads.
// A reset that finds a background job drawing the env's record right now
// (status SPAWN_DRAWING, set by do_spawn_bg) waits for the job to publish
// instead of voiding it and drawing the same permutations again inline: the
// job was queued at least a step earlier and is usually close to done, while an
// inline 40x40 attempt took ~70-80 us of k_post_lean's span in a quarter of
// cfg5's steps (round 5 kernel trace). The wait is bounded (KCfg.draw_wait ticks
// of the 100 MHz clock, by default 2 ms, far beyond a job's ~100 us;
// snake_debug_set("draw_wait_ticks") changes it, e.g. 0 for the test of the
// fallback); after it the claim voids the job as before and the reset draws from
// the env's own state -- right for a job that started from a partial record too:
// the env's state is where that record's failed permutations began, so the reset
// replays them. The voided job may still be drawing; it writes only its own
// queue set's record buffer, which nothing reads until a later job of that set
// (same stream, after it) publishes there, and its final compare-and-swap fails
// against the claim's generation.
__device__ __forceinline__ int claim_reset_mt(const KCfg &c, const snake_state &st, int64_t e, WaveMT &mt,
                                              int lane, uint32_t &cellw)
{
    int v = 0;
    if (lane == 0) {
        uint32_t *wp = reinterpret_cast<uint32_t *>(st.env + e * kEnvRec + ENV_SPAWN);
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        const unsigned long long wait = (unsigned)c.draw_wait;
        if (c.diag && (ld_sc1(wp) & 3u) == SPAWN_DRAWING) DIAG_ADD(g_draw_wait);
        while ((ld_sc1(wp) & 3u) == SPAWN_DRAWING && __builtin_amdgcn_s_memrealtime() - t0 < wait)
            __builtin_amdgcn_s_sleep(8);
        v = (int)atomicAdd(wp, kGenOne);
        if (c.diag && (v & 3) == SPAWN_DRAWING) DIAG_ADD(g_draw_timeout);
    }
    int spw = __shfl(v, 0);
    if ((spw & 3) == SPAWN_DRAWING) spw &= ~3;   // (still drawing: from the env's own state, as for NONE)
    cellw = 0;
    if ((spw & 3) != SPAWN_NONE) {
        const uint32_t *rec = spawn_rec(c, st, e, (spw >> kSpawnBufShift) & (kQSets - 1));
        mt_load_sc1(mt, rec, (int)ld_sc1(rec + kSpawnPos), lane);
        cellw = ld_sc1(rec + kSpawnCells + (lane >> 1));
    } else {
        mt_load(mt, st.mt + e * kMtN, st.env[e * kEnvRec + ENV_MTPOS], lane);
    }
    return spw;
}

// ------------------------------------------------------------------- reset
// SnakeEnv.reset (snake_env.py:131-159): walled grid, S spawn poses =
// permutation(n_cand)[:S] retried until disjoint (:576-589), Snake(idx, coords)
// (core/snake.py:53-74), num_fruits fruit draws, first observation replicated
// over the frame stack. `mt` comes from load_reset_mt: with a ready spawn-ahead
// record the poses are the record's and the draws are already done; a partial
// record continues the retries where the record left them.
// The rest of the reset once the spawn cells are known (lane's cell, lanes <
// S*L): the grid, the snakes, the fruits, the records and the first observation.
__device__ __forceinline__ void reset_paint(const KCfg &c, const snake_state &st, const snake_out &o, int e, WaveMT &mt, uint8_t *lds,
                            int spw, int cell, bool failed, int lane);

template <int MS, int JL>
__device__ void do_reset(const KCfg &c, const snake_state &st, const snake_out &o, int e,
                         WaveMT &mt, uint8_t *lds, int slot, int spw, uint32_t cellw, int lane)
{
    const int spst = spw & 3;
    const int SL = c.S * c.L;
    int cell = -1;
    bool failed = false;
    if (spst == SPAWN_READY) {   // the record's cells (loaded with its key)
        if (lane < SL) cell = (int)((cellw >> (16 * (lane & 1))) & 0xffffu);
    } else {
        // The reference retries forever; a board too crowded for S disjoint spawn
        // poses would hang the wave, so give up after 2^16 permutations and flag
        // the env (env word ENV_FAIL; snake_plan rejects boards where that is
        // likelier than ~1e-6 per reset)
        int q[MS];
        bool ok = false;
        for (int attempt = 0; attempt < (1 << 16) && !ok; attempt++)
            ok = spawn_attempt<MS, JL>(c, st, mt, lds, slot, q, cell, lane);
        failed = !ok;
    }
    reset_paint(c, st, o, e, mt, lds, spw, cell, failed, lane);
}

__device__ __forceinline__ void reset_paint(const KCfg &c, const snake_state &st, const snake_out &o, int e, WaveMT &mt, uint8_t *lds,
                            int spw, int cell, bool failed, int lane)
{
    const int spst = spw & 3;
    uint8_t *frames = lds + c.lds_frames;
    int *org = reinterpret_cast<int *>(lds + c.lds_centers);
    uint16_t *fbuf = reinterpret_cast<uint16_t *>(lds + c.lds_fruit);
    uint8_t *work = frames + (c.fs - 1) * c.grid_stride;
    const int S = c.S, L = c.L, W = c.W, SL = S * L;
    const int sk = lane / L, si = lane - sk * L;
    // make_grid (grid_util.py:14-20), then paint (:138-144)
    for (int x = lane; x < c.HW; x += kWave) {
        const int r = (int)__umulhi((uint32_t)x, c.mag_W), cc = x - r * W;   // x / W
        work[x] = (r == 0 || cc == 0 || r == c.H - 1 || cc == W - 1) ? C_WALL : C_EMPTY;
    }
    wave_sync();
    const int nxt = __shfl(cell, (lane + 1) & 63);
    const int tailcell = __shfl(cell, min(lane + L - 1, 63));
    // the tail queue holds the whole deque (up to 14 directions): entry j =
    // directions[-1-j] = the direction of body cell L-2-j, on lane sk*L + L-2-j
    const int mydir = dir_of_diff(cell - nxt, W);
    const int nq0 = min(L - 1, 14);
    uint32_t tq0 = 0;
    for (int j = 0; j < nq0; j++) tq0 |= (uint32_t)__shfl(mydir, min(sk * L + L - 2 - j, 63)) << (2 * j);
    if (lane < SL) {
        const int v = (si == 0 ? C_HEAD : (si == L - 1 ? C_TAIL : C_BODY)) + 10 * sk;
        work[cell] = (uint8_t)v;
        uint8_t *ring = st.body + ((int64_t)e * S + sk) * c.ring_cap;
        if (si < L - 1) ring[si] = (uint8_t)dir_of_diff(cell - nxt, W);
        if (si == 0) {
            const int hr = (int)__umulhi((uint32_t)cell, c.mag_W), hc = cell - hr * W;
            const int tr = (int)__umulhi((uint32_t)tailcell, c.mag_W), tc = tailcell - tr * W;
            int4 rec;
            rec.x = hr | (hc << 8) | (tr << 16) | (tc << 24);
            rec.y = dir_of_diff(cell - nxt, W) | (1 << 8);
            rec.z = 0 | ((L - 1) << 16);
            // cached directions[-1] (the direction move() pops next)
            rec.w = (int)(tq0 | ((uint32_t)nq0 << 28));
            reinterpret_cast<int4 *>(st.snake)[(int64_t)e * S + sk] = rec;
            const int og = pack_origin(c, hr, hc);
            for (int f = 0; f < c.fs; f++) {
                org[f * kMaxSnakes + sk] = og;
                st.ctr[((int64_t)e * c.fs + f) * S + sk] = (uint16_t)((hr << 8) | hc);
            }
        }
    }
    wave_sync();
    if (!failed) place_fruits_fresh(c, work, mt, c.num_fruits, cell, lane);   // :147-148
    else place_fruits(c, work, mt, c.num_fruits, fbuf, lane);     // (overlapping snakes: count the grid)
    uint8_t *gbase = st.grid + (int64_t)e * c.fs * c.grid_stride;
    const int n16 = c.grid_stride >> 4;
    for (int q = lane; q < n16; q += kWave) {
        const uint4 v = reinterpret_cast<const uint4 *>(work)[q];
        for (int s = 0; s < c.fs; s++) reinterpret_cast<uint4 *>(gbase + s * c.grid_stride)[q] = v;
        for (int s = 0; s < c.fs - 1; s++) reinterpret_cast<uint4 *>(frames + s * c.grid_stride)[q] = v;
    }
    if (lane == 0) {
        int4 er;
        er.x = S; er.y = 0; er.z = c.fs - 1; er.w = mt.pos;
        *reinterpret_cast<int4 *>(st.env + (int64_t)e * kEnvRec) = er;
        // record used up (background: the claim's bumped generation, buffer 0)
        if (c.bg) st.env[(int64_t)e * kEnvRec + ENV_SPAWN] = (int)((((uint32_t)spw >> kSpawnGenShift) + 1u) << kSpawnGenShift);
        else if (spst != SPAWN_NONE) st.env[(int64_t)e * kEnvRec + ENV_SPAWN] = spw & ~3;
        st.env[(int64_t)e * kEnvRec + ENV_FAIL] = failed ? 1 : 0;
        if (failed && o.err) o.err[e] = 2;
    }
    if (lane < 2 * S) reinterpret_cast<uint64_t *>(st.stats)[(int64_t)e * 2 * S + lane] = 0ull;   // _reset_epi_stats
    mt_store(mt, st.mt + (int64_t)e * kMtN, lane);
    wave_sync();
    // (the direct encode: on the reset's critical path the staged row-wise
    // encode's two extra LDS passes cost more than they save)
    encode(c, frames, org, 0, o.obs + (int64_t)e * c.units * 8, lane);
}

// -------------------------------------------------------------------- step
// Copy bytes [0, n) (n % 16 == 0) global -> LDS, 16 B per lane, up to four
// loads in flight per lane before the LDS writes.
__device__ __forceinline__ void stage_to_lds(uint8_t *dst, const uint8_t *src, int n, int lane)
{
    const int n16 = n >> 4;
    const uint4 *s4 = reinterpret_cast<const uint4 *>(src);
    uint4 *d4 = reinterpret_cast<uint4 *>(dst);
    for (int q = lane; q < n16; q += 4 * kWave) {
        const int q1 = q + kWave, q2 = q + 2 * kWave, q3 = q + 3 * kWave;
        const uint4 a = s4[q];
        const uint4 b = q1 < n16 ? s4[q1] : a;
        const uint4 c = q2 < n16 ? s4[q2] : a;
        const uint4 d = q3 < n16 ? s4[q3] : a;
        d4[q] = a;
        if (q1 < n16) d4[q1] = b;
        if (q2 < n16) d4[q2] = c;
        if (q3 < n16) d4[q3] = d;
    }
}

// ---------------------------------------------------------- step: the rules
// k_logic runs SnakeEnv.step up to the observation -- rules, grid update, fruit
// respawn, statistics and outputs -- for E = 64 / MS envs per wave: lane
// (g, k) = snake k of the block's env g, so the per-snake rules of 16 (S <= 4),
// 8 or 4 envs share every instruction and every memory round trip. The new
// frame goes to its ring slot; an env whose episode ended is queued for its
// auto-reset. The wave-wide parts (dying-body erase, fruit respawn) loop over the
// block's envs that need them.
//
// The round-1 inputs of one group (LogicIn, logic_load): env records, snake
// records, actions, running statistics; logic_body runs the group. (A
// persistent form whose waves loaded the next group's inputs, frames
// included, before running the current one measured slower: cfg3 k_logic 24.4
// -> 30.6 us at 8 waves per CU, 42.5 at 4 -- the per-wave latency chain, not
// the loads, sets the kernel's length.)
struct LogicIn {
    int4 er, er2, rec;
    uint4 sv;
    int act;
    uint32_t gate;   // bg: the queue set's finished spawn-kernel count (lane 0)
};

template <int MS, bool BG>
__device__ __forceinline__ void logic_load(const int blk, LogicIn &in)
{
    const KArgs &A = kargs();
    const KCfg &c = A.c;
    const snake_state &st = A.st;
    constexpr int G = MS, E = kWave / MS;
    const int lane = threadIdx.x & (kWave - 1), g = lane / G, k = lane - g * G;
    const int e0 = blk * E, e = e0 + g;
    const int S = c.S;
    const bool env_ok = e < c.N;
    in.er = in.er2 = in.rec = make_int4(0, 0, 0, 0);
    in.sv = make_uint4(0, 0, 0, 0);
    in.act = 0;
    in.gate = 0;
    if (BG && lane == 0) {
        const int *qc = st.resetq + (int64_t)c.qpar * (kNumQ * kQShards * c.q_cap + kQCounters) + kNumQ * kQShards * c.q_cap;
        in.gate = ld_sc1(reinterpret_cast<const uint32_t *>(&qc[kQSpGen * kQSpread]));
    }
    if (env_ok) {
        in.er = *reinterpret_cast<const int4 *>(st.env + (int64_t)e * kEnvRec);
        // loaded whatever the threshold: a step run with spawn-ahead off must
        // still void a record its fruit draws make stale
        in.er2 = *reinterpret_cast<const int4 *>(st.env + (int64_t)e * kEnvRec + 4);
    }
    if (env_ok && k < S) {
        in.rec = reinterpret_cast<const int4 *>(st.snake)[(int64_t)e * S + k];
        in.act = reinterpret_cast<const int8_t *>(A.aux)[(int64_t)e * S + k];
        // the snake's running episode statistics, one 16-byte record (snake_epi_stat)
        in.sv = reinterpret_cast<const uint4 *>(st.stats)[(int64_t)e * S + k];
    }
}

// FU: the fused step (k_step): the stores another wave of the same launch reads
// or writes are write-through (sc1) and drained before the group's done flag
// and the logic-done counter; an env whose episode ended stores nothing its
// auto-reset rewrites (records, statistics, ring words, crop centres, frame):
// the two would race in two XCDs' L2s (k_step, below).
template <int MS, bool BG, bool FU = false>
__device__ __forceinline__ void logic_body(const int blk, const LogicIn &in)
{
    LSTAMP(40);
    const KArgs &A = kargs();
    const KCfg &c = A.c;
    const snake_state &st = A.st;
    const snake_out &o = A.o;
    constexpr int G = MS, E = kWave / MS;
    constexpr uint32_t gmask = (1u << G) - 1u;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds_all[];
    uint8_t *lds = lds_all + (threadIdx.x >> 6) * c.lds_logic;   // (this wave's share of the block's LDS)
    const int lane = threadIdx.x & (kWave - 1), g = lane / G, k = lane - g * G, gb = g * G;
    const int e0 = blk * E, e = e0 + g;
    const int S = c.S, W = c.W, cap = c.ring_cap, fs = c.fs, stride = c.grid_stride;
    const int n16 = stride >> 4;
    const bool env_ok = e < c.N;
    const bool isn = env_ok && k < S;
    uint8_t *work = lds + g * stride;                      // this env's grid being stepped
    uint16_t *fbuf = reinterpret_cast<uint16_t *>(lds + E * stride);
    // per-env respawn scratch: G * kRespawnT tempered raws, G chosen cells
    uint32_t *rawbuf = reinterpret_cast<uint32_t *>(lds + E * stride + 2 * kMaxFruits) + g * (G * kRespawnT);
    uint16_t *cellbuf = reinterpret_cast<uint16_t *>(lds + E * stride + 2 * kMaxFruits + E * G * kRespawnT * 4) + g * G;
    // this step's queue set and its counters (zero between steps: the last
    // k_autoreset worker re-zeroes them; the spawn counters of a background
    // step, the next step's k_autoreset)
    int *qb = st.resetq + (int64_t)c.qpar * (kNumQ * kQShards * c.q_cap + kQCounters);
    int *qcnt = qb + kNumQ * kQShards * c.q_cap;
    auto gbits = [&](unsigned long long m) -> uint32_t { return (uint32_t)(m >> gb) & gmask; };

    // ---- the round-1 inputs (logic_load)
    const int4 er = in.er, er2 = in.er2, rec = in.rec;
    const uint4 sv = in.sv;
    const int act = in.act;
    const int spst = er2.x & 3;   // ENV_SPAWN
    uint4 *sp = reinterpret_cast<uint4 *>(st.stats) + (int64_t)e * S + k;
    const int alive0 = er.x, eplen = er.y, cur = er.z, mtpos = er.w;
    // stage the E current frames (env g's at lds + g * stride): eight 16-B loads
    // in flight per lane before the LDS writes (a load-wait-write loop pays one
    // memory round trip per 64 chunks). Branch-free: tail lanes re-stage the last
    // chunk, the missing envs of a partial block stage the last env. With one
    // frame the slot is 0 and the loads do not wait for the env records.
    auto stage = [&](auto one) {
        constexpr bool ONE = decltype(one)::value;
        const uint4 *src = reinterpret_cast<const uint4 *>(st.grid);
        uint4 *d4 = reinterpret_cast<uint4 *>(lds);
        const int nq = E * n16;
        // (vector values, not arrays: the arrays were demoted to scratch)
        typedef uint32_t v32u __attribute__((ext_vector_type(32)));
        typedef int v8i __attribute__((ext_vector_type(8)));
        for (int q0 = 0; q0 < nq; q0 += 8 * kWave) {   // uniform trip count (the __shfl)
            v32u v;
            v8i qq;
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const int q = min(q0 + u * kWave + lane, nq - 1);
                const int gg = fdiv((uint32_t)q, c.mag_n16, n16), off = q - gg * n16;
                const int cg = ONE ? 0 : __shfl(cur, gg * G);
                const int64_t ee = min(e0 + gg, c.N - 1);
                const uint4 x = src[(ee * c.ring_bytes + (int64_t)cg * stride) / 16 + off];
                v[4 * u] = x.x; v[4 * u + 1] = x.y; v[4 * u + 2] = x.z; v[4 * u + 3] = x.w;
                qq[u] = q;
            }
#pragma unroll
            for (int u = 0; u < 8; u++) d4[qq[u]] = make_uint4(v[4 * u], v[4 * u + 1], v[4 * u + 2], v[4 * u + 3]);
        }
    };
    if (fs == 1) stage(std::true_type{});
    else stage(std::false_type{});
    LSTAMP(51);
    // keep the statistics loads up here with the others (the compiler would sink
    // them to their first use, deep in the step, and pay a full memory latency there)
    __asm__ volatile("" ::"v"(sv.x), "v"(sv.y), "v"(sv.z), "v"(sv.w));
    LSTAMP(52);
    double s0 = __hiloint2double((int)sv.y, (int)sv.x);
    uint32_t s1 = sv.z, s2 = sv.w & 0xffffu, s3 = sv.w >> 16;
    const int ncur = (fs == 1) ? 0 : (cur + 1 == fs ? 0 : cur + 1);
    int hr = rec.x & 255, hc = (rec.x >> 8) & 255, tr = (rec.x >> 16) & 255, tc = (rec.x >> 24) & 255;
    int dir = rec.y & 3, alive = (rec.y >> 8) & 1;
    int rh = rec.z & 0xffff, rl = (rec.z >> 16) & 0xffff;
    // Direction deque (body ring) traffic: the ring word holding the head is
    // written once per 4 pushes (pending directions in rec.y bits 16-23, 2 bits
    // per byte offset), and the tail end is read as aligned 8-byte chunks into a
    // queue in rec.w (entry 0 = directions[-1], then directions[-2], ...; count
    // in bits 28-31). One byte store and one line fetch per snake and step
    // were the largest share of k_logic's traffic. A queue whose count equals
    // rl holds the whole deque (every snake of up to 14 directions, i.e. all
    // fresh ones): it is kept whole by appending each step's new head direction
    // and never refills from the ring -- a refill every 2-3 steps for a short
    // snake, in the same step for every env after a reset of all of them.
    uint32_t tq = (uint32_t)rec.w;
    const int tdir = (int)(tq & 3u);          // directions[-1] (core/snake.py:103)
    int hbuf = (rec.y >> 16) & 255;

    // snake_env.py:318-330 heading + target cell per alive snake
    const bool mv0 = isn && alive;
    int nd = dir;
    if (c.observer == 0) {                 // _next_direction :598-608 (0 keep, 1 left, 2 right)
        nd = (act == 1) ? ((dir + 3) & 3) : ((act == 2) ? ((dir + 1) & 3) : dir);
    } else if (dir_dr(dir) == 0) {         // _next_direction_global :610-632
        nd = (act == 3) ? 2 : ((act == 4) ? 0 : dir);
    } else {
        nd = (act == 1) ? 3 : ((act == 2) ? 1 : dir);
    }
    // an invalid action of an alive snake raises KeyError in the reference before
    // anything changes: that env is left untouched (only err/ep_done are written)
    const bool bad = gbits(__ballot(mv0 && c.observer == 0 && (act < 0 || act > 2))) != 0u;
    const bool live = isn && !bad;
    const bool mv = mv0 && !bad;
    if (mv) dir = nd;
    const int ncell = mv ? (hr + dir_dr(dir)) * W + hc + dir_dc(dir) : -1 - lane;
    wave_sync();
    LSTAMP(41);

    // _check_collision :521-544 -- groups of snakes with the same target cell
    // (lanes k >= S hold no snake: their ncell -1 - lane matches nothing)
    int cnt = 0;
    bool lower = false;
    unroll<G>([&](auto J) {
        const bool same = gsel<G, J>(ncell) == ncell;
        cnt += same;
        lower |= same && J < k;
    });
    const bool leader = mv && !lower;
    const int v = mv ? work[ncell] : 0;
    const int vid = div10(v), cv = v - 10 * vid;
    const bool deadly = mv && (cnt > 1 || cv == C_WALL || cv == C_BODY || cv == C_HEAD);
    const bool eat = mv && !deadly && cv == C_FRUIT;
    // every target group on a fruit cell counts once: an eater, or a head-on there
    // (the fruit stays and one more spawns)
    const int fruit_taken = __popc(gbits(__ballot(leader && cv == C_FRUIT)));
    // kill credit: one per deadly group on a BODY/HEAD cell, to its owner (self too)
    const int owner = (leader && deadly && (cv == C_BODY || cv == C_HEAD)) ? vid : -1;
    int kills = 0;
    unroll<G>([&](auto J) { kills += gsel<G, J>(owner) == k; });   // (owner -1 off the snakes)
    int alive_snakes = alive0 - __popc(gbits(__ballot(deadly)));            // :334
    bool death = deadly;
    // :338-346 a fruit eater's tail does not move: snakes entering it die (again)
    const int etail = eat ? tr * W + tc : -2;
    bool hit = false;
    unroll<G>([&](auto J) {   // (off the snakes: etail -2, ncell -1 - lane)
        const int ej = gsel<G, J>(etail), nj = gsel<G, J>(ncell);
        hit |= mv && ej == ncell;
        kills += (eat && nj == etail) ? 1 : 0;
    });
    alive_snakes -= __popc(gbits(__ballot(hit)));
    death |= hit;
    alive = mv && !death;
    const uint32_t am = gbits(__ballot(isn && alive));
    const bool win = alive_snakes == 1 && S > 1 && am && k == __ffs(am) - 1;

    // episode end (:391-394 truncation, coop any-done) is known here: claim the
    // auto-reset queue slots now, one atomic per wave on this block's shard, so the
    // atomic's round trip overlaps the rest of the step
    const int eplen1 = eplen + 1;
    const int dn = !alive;
    int fd = ((double)eplen1 >= c.max_steps) ? 1 : dn;
    const uint32_t done_m = gbits(__ballot(isn && fd));
    const uint32_t all_m = (1u << S) - 1u;
    const bool ep_end = !bad && (c.coop ? (done_m != 0u) : (done_m == all_m));
    if (c.coop && ep_end) fd = 1;
    // (autoreset 2: every env, gym 0.23.1's reset after every step, except an
    // env rejected for an invalid action: k_encode encodes its unchanged state)
    const unsigned long long qm = c.autoreset ? __ballot(env_ok && k == 0 && !bad && (ep_end || c.autoreset == 2))
                                              : 0ull;
    const int shard = blk % kQShards;
    int qbase = 0;
    if (qm && lane == 0) qbase = atomicAdd(&qcnt[shard * kQSpread], __popcll(qm));

    // rewards, fp64 in the reference order (:354-370)
    const bool counted = death || alive;   // not previously dead
    double rew = 0.0;
    if (counted) {
        double r = c.rt * (double)alive;
        r += c.rf * (double)eat;
        r += c.rl * (double)death;
        r += c.rk * (double)kills;
        r += c.rw * (double)win;
        rew = r;
    }

    // ---- the step's second round of memory accesses, all issued here: their
    // addresses are known once the rules are, and in program order each group
    // cost the wave a memory round trip of its own. The tail-queue refill of a
    // snake that empties its queue (at the head slot after this step's push),
    // the first 16 body directions of a dying snake, the fruit-respawn raw words
    // of an env that needs a fruit, and the spawn-ahead queue claims.
    // per env (all G lanes of the group, snake or not): a fruit respawn
    const bool need = env_ok && !bad && fruit_taken > 0;
    // spawn-ahead (include/snake_env.h): a draw from the MT state voids the env's
    // record; an env near its episode end without a ready record is queued for
    // one attempt of its next reset (this step's k_autoreset workers). Claimed
    // as if every respawn drew (a queued env whose record stays ready is skipped
    // by its job); the status word written below is the exact one.
    // urgent (at most one live snake: the reset is likely next) and other jobs
    const bool urgent = __popc(am) <= 1;
    // (background: only into a queue set its spawn kernels have finished with)
    const bool set_free = !BG || (uint32_t)bcast((int)in.gate, 0) == c.spawn_gate;
    if (BG && c.diag && !set_free && lane == 0) DIAG_ADD(g_gate_shut);
    const bool spawn_q = c.spawn_thr >= 0 && set_free && env_ok && !bad && !ep_end &&
                         (need ? true : spst < SPAWN_READY) && __popc(am) <= c.spawn_thr;   // (DRAWING: a job has it)
    const unsigned long long pm = __ballot(spawn_q && urgent && k == 0);
    const unsigned long long pn = __ballot(spawn_q && !urgent && k == 0);
    int pbase = 0, nbase = 0;
    if (pm && lane == 0) pbase = atomicAdd(&qcnt[(kQShards + shard) * kQSpread], __popcll(pm));
    if (pn && lane == 0) nbase = atomicAdd(&qcnt[(2 * kQShards + shard) * kQSpread], __popcll(pn));

    uint8_t *ring = st.body + ((int64_t)e * S + k) * cap;
    const uint32_t tcnt0 = tq >> 28;
    const bool tfull = (int)tcnt0 == rl;   // the queue holds the whole deque
    const bool refill = alive && !eat && tcnt0 == 1u && !tfull;
    const int rt1 = (((rh - 1) & (cap - 1)) + rl - 1) & (cap - 1), rbase = rt1 & ~7;
    uint64_t rchunk = 0;
    if (refill) rchunk = *reinterpret_cast<const uint64_t *>(ring + rbase);
    const bool dying = isn && death;
    // (the two aligned 16-byte ring chunks that hold positions rh .. rh + 15)
    uint4 dc0 = make_uint4(0, 0, 0, 0), dc1 = make_uint4(0, 0, 0, 0);
    if (dying) {
        dc0 = *reinterpret_cast<const uint4 *>(ring + (rh & (cap - 16)));
        dc1 = *reinterpret_cast<const uint4 *>(ring + ((rh + 16) & (cap - 16)));
    }
    // the next G * kRespawnT raw words of the stream; past the key's end they
    // are words of the next key, computed from the old one (new[j] for j < 227
    // needs old[j], old[j+1] and old[j+397] only): the twist is left pending in
    // the stored position (> 624), every MT consumer applies it
    const bool room = mtpos + G * kRespawnT <= kMtN + 226;
    // (issued for every env right after the staging instead, before the rules
    // say which envs eat: cfg3 k_logic 24.0 -> 26.0 us, cfg4 20.0 -> 19.4,
    // round 5, profiles/r05_ab_raw_early.jsonl)
    uint32_t raws[kRespawnT];
    {
        const uint32_t *key = st.mt + (int64_t)e * kMtN;
#pragma unroll
        for (int t = 0; t < kRespawnT; t++) {
            const int pw = mtpos + t * G + k;
            raws[t] = 0u;
            if (need && room) {
                if (pw < kMtN) {
                    raws[t] = key[pw];
                } else {
                    const int j = pw - kMtN;
                    raws[t] = mt_mix(key[j], key[j + 1], key[j + 397]);
                }
            }
        }
    }
    // _update_grid in two phases. Phase 1: every tail that leaves its cell is
    // cleared if it still holds this snake's TAIL, and every dying snake's tail
    // if it is still this snake's; phase 2: BODY at the old head, HEAD at the
    // new head, TAIL at the new tail. Phase-2 cells are pairwise distinct and a
    // phase-1 cell is rewritten in phase 2 only by a snake entering that tail,
    // which is what the reference's index-ordered updates produce.
    LSTAMP(42);
    // One frame (fs == 1): the slot is rewritten in place, so only the 16-byte
    // chunks this step writes go back to it (bit q of dm = chunk q of the frame,
    // frames of up to 64 chunks); the commit below ORs the group's masks
    uint64_t dm = 0;
    auto dirty = [&](int cell) { dm |= 1ull << (((unsigned)cell >> 4) & 63u); };
    const int pt = tr * W + tc;
    if (alive && !eat) {
        if (work[pt] == C_TAIL + 10 * k) work[pt] = C_EMPTY;
        dirty(pt);
    }
    if (isn && death) {
        if (div10(work[pt]) == k) work[pt] = C_EMPTY;
        dirty(pt);
    }
    wave_sync();
    int nhr = hr, nhc = hc, ntr = tr, ntc = tc;
    if (alive) {
        work[hr * W + hc] = (uint8_t)(C_BODY + 10 * k);
        dirty(hr * W + hc);
        nhr = hr + dir_dr(dir);
        nhc = hc + dir_dc(dir);
        rh = (rh - 1) & (cap - 1);                                   // directions.appendleft
        const int ho = rh & 3;
        hbuf = (hbuf & ~(3 << (2 * ho))) | (dir << (2 * ho));
        const int hfull = hbuf;                                      // the head word's directions
        if (ho == 0) {                                               // the head word is complete
            if (!FU || !ep_end)
                *reinterpret_cast<uint32_t *>(ring + rh) = (uint32_t)(hbuf & 3) | ((uint32_t)(hbuf >> 2 & 3) << 8) |
                                                           ((uint32_t)(hbuf >> 4 & 3) << 16) |
                                                           ((uint32_t)(hbuf >> 6 & 3) << 24);
            hbuf = 0;
        }
        if (!eat) {                                                  // directions.pop()
            ntr = tr + dir_dr(tdir);
            ntc = tc + dir_dc(tdir);
            const uint32_t cnt = (tq >> 28) - 1u;
            tq = ((tq & 0x0fffffffu) >> 2) | (cnt << 28);
            if (tfull) {
                tq = (tq & 0x0fffffffu) | ((uint32_t)dir << (2 * cnt)) | ((cnt + 1u) << 28);   // the new directions[0]
            } else if (cnt == 0u) {
                // refill from the chunk holding the new directions[-1] (position t):
                // t, t-1, .. down to the chunk start, but not below the head (the
                // positions past it are free ring slots); pending head-word bytes
                // come from the head word's directions
                const int t = rt1, base = rbase;   // (t = rh + rl - 1 with the new rh)
                const uint64_t q = rchunk;
                const int n = min(t - base + 1, ((t - rh) & (cap - 1)) + 1);
                uint32_t nq = 0;
                for (int j = 0; j < n; j++) {
                    const int p = t - j;
                    int d = (int)(q >> (8 * (p - base))) & 3;
                    // (the chunk was read before this step's head-word store)
                    if ((p >> 2) == (rh >> 2) && p >= rh) d = (hfull >> (2 * (p & 3))) & 3;
                    nq |= (uint32_t)d << (2 * j);
                }
                tq = nq | ((uint32_t)n << 28);
            }
        } else {
            if (tfull && tcnt0 < 14u)   // (a 15th entry does not fit: from then on the ring refills it)
                tq = (tq & 0x0fffffffu) | ((uint32_t)dir << (2 * tcnt0)) | ((tcnt0 + 1u) << 28);
            rl++;
        }
        work[nhr * W + nhc] = (uint8_t)(C_HEAD + 10 * k);
        work[ntr * W + ntc] = (uint8_t)(C_TAIL + 10 * k);
        dirty(nhr * W + nhc);
        dirty(ntr * W + ntc);
    }
    wave_sync();
    // draw(grid, coords, EMPTY) of each dying snake's head and body (the tail was
    // handled above): coords = head - prefix sums of the direction deque
    // (core/snake.py:86-94). Every dying snake walks its own body on its lane, 16
    // ring bytes fetched per memory round trip.
    LSTAMP(43);
    if (dying) {
        const uint8_t *rk = ring;
        int br = hr, bc = hc;
        work[br * W + bc] = C_EMPTY;
        dirty(br * W + bc);
        const int n = rl - 1;
        for (int m0 = 0; m0 < n; m0 += 16) {
            int d[16];
#pragma unroll
            for (int t = 0; t < 16; t++) {
                if (m0 == 0) {   // from the two chunks loaded with the second round
                    const int x = (rh & 15) + t;
                    const uint32_t w = x < 16 ? (x < 8 ? (x < 4 ? dc0.x : dc0.y) : (x < 12 ? dc0.z : dc0.w))
                                              : (x < 24 ? (x < 20 ? dc1.x : dc1.y) : (x < 28 ? dc1.z : dc1.w));
                    d[t] = t < n ? (int)((w >> (8 * (x & 3))) & 255u) : 0;
                } else {
                    d[t] = (m0 + t < n) ? rk[(rh + m0 + t) & (cap - 1)] : 0;
                }
            }
            if (m0 == 0 && (rh & 3) != 0) {                          // the pending head-word bytes
#pragma unroll
                for (int t = 0; t < 3; t++)
                    if (t < 4 - (rh & 3)) d[t] = (hbuf >> (2 * ((rh & 3) + t))) & 3;
            }
#pragma unroll
            for (int t = 0; t < 16; t++) {
                if (m0 + t < n) {
                    br -= dir_dr(d[t]);
                    bc -= dir_dc(d[t]);
                    work[br * W + bc] = C_EMPTY;
                    dirty(br * W + bc);
                }
            }
        }
    }
    wave_sync();

    LSTAMP(44);
    // fruit respawn (:376-379, random_empty_coords grid_util.py:126-133). Fast
    // path, every env at once on its own G lanes: the draws read the next
    // G * kRespawnT raw words of the env's key straight from memory (no twist
    // needed, the key is not rewritten); the empties are counted per lane over a
    // slice of the grid and the v-th one found by the lane whose slice holds it.
    int mtpos_new = mtpos;
    bool mt_slow = false;
    // (per env, all G lanes of the group, snake or not: the empties are counted by all)
    bool fast_done = false;
    if (__ballot(need)) {
        // lane k of the group counts the empty cells of its slice of 16-byte
        // chunks (bytes past the grid count as occupied)
        const int HW = c.HW, nc = (HW + 15) >> 4, cpl = (nc + G - 1) / G;
        const int q0 = min(nc, k * cpl), q1 = min(nc, q0 + cpl);
        auto chunk = [&](int q) {
            uint4 x = reinterpret_cast<const uint4 *>(work)[q];
            if (q == nc - 1 && (HW & 15)) {
                const int r = HW & 15;
                x.x |= r >= 4 ? 0u : 0xffffffffu << (8 * r);
                x.y |= r >= 8 ? 0u : (r <= 4 ? 0xffffffffu : 0xffffffffu << (8 * (r - 4)));
                x.z |= r >= 12 ? 0u : (r <= 8 ? 0xffffffffu : 0xffffffffu << (8 * (r - 8)));
                x.w |= r <= 12 ? 0xffffffffu : 0xffffffffu << (8 * (r - 12));
            }
            return x;
        };
        int cnt = 0;
        if (need) {
            for (int q = q0; q < q1; q++) {
                const uint4 x = chunk(q);
                cnt += zero_bytes(x.x) + zero_bytes(x.y) + zero_bytes(x.z) + zero_bytes(x.w);
            }
        }
        const int incl = gscan<G>(cnt, k);
        const int excl = incl - cnt;
        const int Etot = gsel<G, G - 1>(incl);
        const uint32_t rng = (uint32_t)(Etot - 1), rmask = gen_mask(rng);
        // rng == 0 draws nothing (randint(0, 1) consumes no raw word)
        const bool draws = need && Etot > 0 && rng != 0;
        // the raw words were loaded with the second round (above)
        uint32_t accm = 0;
#pragma unroll
        for (int t = 0; t < kRespawnT; t++) {
            const uint32_t raw = (draws && room) ? raws[t] : 0u;
            const uint32_t tv = temper(raw) & rmask;
            rawbuf[t * G + k] = tv;
            accm |= gbits(__ballot(draws && room && tv <= rng)) << (t * G);
        }
        const bool fast = need && Etot > 0 && (!draws || (room && __popc(accm) >= fruit_taken));
        wave_sync();
        uint32_t am2 = accm;
        int used = 0;
        for (int d = 0; d < MS; d++) {
            const bool act_d = fast && d < fruit_taken;
            int v = 0;
            if (act_d && draws) {
                const int p = __ffs(am2) - 1;
                am2 &= am2 - 1u;
                v = (int)rawbuf[p];
                used = p + 1;
            }
            if (act_d && v >= excl && v < excl + cnt) {      // this lane's slice holds it
                int need_n = v - excl, x = -1;
                for (int q = q0; q < q1 && x < 0; q++) {
                    const uint4 y4 = chunk(q);
                    const int z0 = zero_bytes(y4.x), z1 = zero_bytes(y4.y), z2 = zero_bytes(y4.z), z3 = zero_bytes(y4.w);
                    if (need_n >= z0 + z1 + z2 + z3) {
                        need_n -= z0 + z1 + z2 + z3;
                        continue;
                    }
                    // the dword, then the byte
                    int dw = 0;
                    uint32_t y = y4.x;
                    if (need_n >= z0) { need_n -= z0; dw = 1; y = y4.y;
                        if (need_n >= z1) { need_n -= z1; dw = 2; y = y4.z;
                            if (need_n >= z2) { need_n -= z2; dw = 3; y = y4.w; } } }
                    for (int b = 0; b < 4; b++) {
                        if (((y >> (8 * b)) & 255u) == 0u) {
                            if (need_n == 0) { x = 16 * q + 4 * dw + b; break; }
                            need_n--;
                        }
                    }
                }
                cellbuf[d] = (uint16_t)x;
            }
        }
        wave_sync();
        if (fast && k < fruit_taken) {
            work[cellbuf[k]] = C_FRUIT;
            dirty(cellbuf[k]);
        }
        if (fast && draws) mtpos_new = mtpos + used;
        fast_done = fast;
        wave_sync();
    }
    // the rest (a twist needed, or too few accepts among the prefetched raws), one
    // env at a time with the whole wave
    unsigned long long fm = __ballot(need && !fast_done && k == 0);
    if (c.diag && need && !fast_done && k == 0) {
        if (!room) DIAG_ADD(g_resp_slow);
        else DIAG_ADD(g_resp_slow2);
    }
    while (fm) {
        const int L = __ffsll((long long)fm) - 1;
        fm &= fm - 1;
        const int gg = L / G;
        const int64_t ee = e0 + gg;
        WaveMT mt;
        mt_load(mt, st.mt + ee * kMtN, bcast(mtpos, L), lane);
        place_fruits(c, lds + gg * stride, mt, bcast(fruit_taken, L), fbuf, lane);
        if constexpr (FU) {   // (a reset or spawn-ahead job of this launch may read the key)
#pragma unroll
            for (int t = 0; t < 10; t++)
                if (64 * t + lane < kMtN) st_sc1(st.mt + ee * kMtN + 64 * t + lane, mt.w[t]);
        } else {
            mt_store(mt, st.mt + ee * kMtN, lane);
        }
        if (g == gg) { mtpos_new = mt.pos; mt_slow = true; dm = ~0ull; }
    }
    // a draw from the MT state voids the env's spawn-ahead record
    const bool drew = mt_slow || mtpos_new != mtpos;
    // (a draw bumps the record's generation: a background attempt started from the
    // old state (k_spawn) then fails its final compare-and-swap, or, if that landed
    // first, is overwritten here; so with bg every draw writes the word)
    const bool spw_wr = drew && (BG || spst != SPAWN_NONE);
    if (c.diag && drew && spst == SPAWN_READY && k == 0) DIAG_ADD(g_spawn_void);
    const uint32_t spw1 = drew ? (((uint32_t)er2.x >> kSpawnGenShift) + 1u) << kSpawnGenShift : (uint32_t)er2.x;

    LSTAMP(45);
    // episode statistics (:385-389), truncation (:391-394), rank/info (:396-412)
    if (isn) {   // (steps/fruits/kills: the reference's msk * x sums, held as integers)
        const double msk = 1.0 - (double)dn;
        s0 = s0 + msk * rew;
        s1 += dn ? 0u : 1u;
        s2 += (!dn && counted) ? (uint32_t)eat : 0u;
        s3 += (!dn && counted) ? (uint32_t)kills : 0u;
    }
    if (isn) {   // an env rejected for an invalid action reports reward 0, not done
        o.rew[(int64_t)e * S + k] = live ? rew : 0.0;
        o.done[(int64_t)e * S + k] = (uint8_t)(live ? fd : 0);
    }
    if (env_ok && k == 0) {
        o.ep_done[e] = ep_end ? 1 : 0;
        o.err[e] = bad ? 1 : 0;
    }
    LSTAMP(48);
    if (qm) {            // queue the auto-resets in the slots claimed above
        const int base = bcast(qbase, 0);
        if ((qm >> lane) & 1ull) {
            int *qp = qb + shard * c.q_cap + base + mbcnt64(qm);
            if constexpr (FU) st_sc1(reinterpret_cast<uint32_t *>(qp), (uint32_t)e);
            else *qp = e;
        }
    }
    // and the spawn-ahead jobs (background: with the generation they were queued at)
    const int pent = BG ? (int)((uint32_t)e | ((spw1 >> kSpawnGenShift) << (32 - kQGenBits))) : e;
    if (pm) {
        const int base = bcast(pbase, 0);
        if ((pm >> lane) & 1ull) {
            int *qp = qb + (kQShards + shard) * c.q_cap + base + mbcnt64(pm);
            if constexpr (FU) st_sc1(reinterpret_cast<uint32_t *>(qp), (uint32_t)pent);
            else *qp = pent;
        }
    }
    if (pn) {
        const int base = bcast(nbase, 0);
        if ((pn >> lane) & 1ull) {
            int *qp = qb + (2 * kQShards + shard) * c.q_cap + base + mbcnt64(pn);
            if constexpr (FU) st_sc1(reinterpret_cast<uint32_t *>(qp), (uint32_t)pent);
            else *qp = pent;
        }
    }
    if (env_ok && k == 0 && !bad && spw_wr) {
        if (BG) atomicExch(reinterpret_cast<uint32_t *>(st.env + (int64_t)e * kEnvRec + ENV_SPAWN), spw1);
        else if (FU) st_sc1(reinterpret_cast<uint32_t *>(st.env + (int64_t)e * kEnvRec + ENV_SPAWN), spw1);
        else st.env[(int64_t)e * kEnvRec + ENV_SPAWN] = (int)spw1;
    }
    LSTAMP(49);
    int rank = 1;
    unroll<G>([&](auto J) { rank += (J < S && gsel<G, J>(s0) > s0) ? 1 : 0; });
    if (isn && ep_end) {   // the episode summary where it ended (nothing stored elsewhere:
                           // ~1.5 % of the envs at cfg3, 9.4 of k_logic's MB per step)
        o.rank[(int64_t)e * S + k] = rank;
        double *es = o.ep_stats + (int64_t)e * 4 * S;
        es[k] = s0; es[S + k] = (double)s1;
        es[2 * S + k] = (double)s2; es[3 * S + k] = (double)s3;
    }
    if (ep_end) { s0 = 0.0; s1 = s2 = s3 = 0u; }                   // _reset_epi_stats
    // a snake dead before this step keeps its statistics, record and (one frame)
    // crop centre: no stores for it
    if (live && (counted || ep_end) && !(FU && ep_end)) {
        const unsigned long long sb = (unsigned long long)__double_as_longlong(s0);
        *sp = make_uint4((uint32_t)sb, (uint32_t)(sb >> 32), s1, (s2 & 0xffffu) | (s3 << 16));
    }

    LSTAMP(46);
    // commit the new frames into their ring slots (one frame: the chunks the
    // step wrote, in place); records; crop centres
    {
        uint4 *dst = reinterpret_cast<uint4 *>(st.grid);
        const uint4 *s4 = reinterpret_cast<const uint4 *>(lds);
        const bool inplace = SNAKE_LOGIC_DIRTY && fs == 1 && n16 <= 64;
        uint32_t dlo = ~0u, dhi = ~0u;
        if (inplace) {
            dlo = dhi = 0u;
            unroll<G>([&](auto J) {
                dlo |= (uint32_t)gsel<G, J>((int)(uint32_t)dm);
                dhi |= (uint32_t)gsel<G, J>((int)(uint32_t)(dm >> 32));
            });
        }
        if (SNAKE_LOGIC_COMMIT_GROUP && inplace) {
            // each env's group commits its own dirty chunks: lane k of the group
            // the set bits k, k + G, k + 2G, ... of the group's mask (no
            // cross-lane moves per chunk, ~3 passes instead of E * n16 / 64)
            // (only the frame's n16 chunks: a full-wave fruit draw marks all 64)
            const uint64_t valid = n16 >= 64 ? ~0ull : (1ull << n16) - 1ull;
            uint64_t m = (env_ok && !bad && !(FU && ep_end)) ? (((uint64_t)dhi << 32) | dlo) & valid : 0ull;
            for (int j = 0; j < k; j++) m &= m - 1ull;
            uint4 *de = dst + (int64_t)e * (c.ring_bytes / 16);   // (one frame: slot 0)
            const uint4 *se = s4 + g * n16;
            while (m) {
                const int off = __ffsll((long long)m) - 1;
                if constexpr (FU) st_sc1_128(de + off, se[off]);
                else de[off] = se[off];
#pragma unroll
                for (int j = 0; j < G; j++) m &= m - 1ull;
            }
        } else
        for (int q0 = 0; q0 < E * n16; q0 += kWave) {
            const int q = q0 + lane, gg = min(fdiv((uint32_t)q, c.mag_n16, n16), E - 1);
            const int off = q - gg * n16;
            const int ng = __shfl(ncur, gg * G);
            const int bg = __shfl((int)(bad || (FU && ep_end)), gg * G);
            const uint32_t ml = (uint32_t)__shfl((int)dlo, gg * G), mh = (uint32_t)__shfl((int)dhi, gg * G);
            const bool wrote = ((off < 32 ? ml >> off : mh >> (off & 31)) & 1u) != 0u;
            if (q < E * n16 && e0 + gg < c.N && !bg && wrote) {
                uint4 *d = dst + ((int64_t)(e0 + gg) * c.ring_bytes + (int64_t)ng * stride) / 16 + off;
                if constexpr (FU) st_sc1_128(d, s4[q]);   // (the encodes read it in this launch)
                else *d = s4[q];
            }
        }
    }
    // crop centre = the own HEAD cell: the new head while alive, (0,0) when dead
    const int chr = alive ? nhr : 0, chc = alive ? nhc : 0;
    if (env_ok && k == 0 && !bad) {
        int4 ner;
        ner.x = alive_snakes; ner.y = eplen1; ner.z = ncur; ner.w = mtpos_new;
        // (FU: this env's auto-reset in this launch reads the MT position)
        if constexpr (FU) st_sc1_128(st.env + (int64_t)e * kEnvRec, make_uint4(ner.x, ner.y, ner.z, ner.w));
        else *reinterpret_cast<int4 *>(st.env + (int64_t)e * kEnvRec) = ner;
    }
    if (live && (counted || fs > 1) && !(FU && ep_end)) st.ctr[((int64_t)e * fs + ncur) * S + k] = (uint16_t)((chr << 8) | chc);
    if constexpr (FU) {
        // the encodes' hand-off record of env e (k_step): the slot to encode,
        // whether the env auto-resets (its reset writes the observation), the S
        // <= 4 crop centres (the own head, (0,0) when dead; an env rejected for
        // an invalid action keeps its slot and heads)
        const int aw = bad ? (isn && ((rec.y >> 8) & 1)) : alive;
        const int cv2 = aw ? (bad ? (hr << 8) | hc : (chr << 8) | chc) : 0;
        const int c0 = gsel<G, 0>(cv2), c1 = gsel<G, 1>(cv2), c2 = gsel<G, 2>(cv2), c3 = gsel<G, 3>(cv2);
        if (env_ok && k == 0) {
            const uint32_t slot = bad ? (uint32_t)cur : (uint32_t)ncur;
            st_sc1_128(st.resetq + c.fu_hoff + 4 * (int64_t)e,
                       make_uint4(slot | ((ep_end && !bad) ? 256u : 0u), (uint32_t)(c0 & 0xffff) | ((uint32_t)c1 << 16),
                                  (uint32_t)(c2 & 0xffff) | ((uint32_t)c3 << 16), 0u));
        }
    }
    if (live && counted && !(FU && ep_end)) {
        int4 nrec;
        nrec.x = nhr | (nhc << 8) | (ntr << 16) | (ntc << 24);
        nrec.y = dir | (alive << 8) | (hbuf << 16);
        nrec.z = rh | (rl << 16);
        nrec.w = (int)tq;                 // entry 0 = the new directions[-1]
        reinterpret_cast<int4 *>(st.snake)[(int64_t)e * S + k] = nrec;
    }
    if constexpr (FU) {
        // publish (MI355X_MICROARCH.md, inter-workgroup visibility, R1): every
        // write-through store drained, then the group's done flag (encodes) and
        // the sharded logic-done count (reset workers)
        __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) {
            st_sc1(reinterpret_cast<uint32_t *>(st.resetq + c.fu_done) + blk, c.epoch);
            atomicAdd(reinterpret_cast<unsigned *>(st.resetq + c.fu_ldone) + (blk % kQShards) * kQSpread, 1u);
        }
    }
    LSTAMP(47);
}

// WPB waves per workgroup, each an independent group of envs (no barrier):
// fewer, larger workgroups for the dispatcher.
// BG: background spawn-ahead (KCfg.bg), its queue-set gate and status-word
// atomics; the in-step form carries none of it
template <int MS, int WPB, bool BG>
__global__ void __launch_bounds__(64 * WPB) k_logic(const KArgs)
{
    WTIME(0);
    const int blk = (int)blockIdx.x * WPB + (int)(threadIdx.x >> 6);
    if (blk * (kWave / MS) >= kargs().c.N) return;
    LogicIn in;
    logic_load<MS, BG>(blk, in);
    logic_body<MS, BG>(blk, in);
    WTIME(1);
}


// ------------------------------------------------------- spawn-ahead records
// Spawn-ahead job of env e (include/snake_env.h snake_step): one permutation
// attempt of its next reset, from its MT state or its partial record, into the
// record. k_logic queues only envs with no ready record whose reset is not this
// step, so nothing else touches the env's MT state or record meanwhile.
// The status word spw is the one the attempt started under (generation kept);
// a background job publishes with a compare-and-swap against it (k_spawn).
// The record goes to buffer nb. Background (k_spawn, BG): write-through stores,
// drained, then published with a compare-and-swap against spw.
// The spawn cells (lane < S*L: `cell`, from spawn_attempt) are stored as u16
// pairs, lanes 2m and 2m + 1 in word m, so a reset reads them with the key.
template <bool BG = false>
__device__ void store_spawn_record(const KCfg &c, const snake_state &st, int e, const WaveMT &mt, bool ok,
                                   int cell, int lane, uint32_t spw, int nb = 0)
{
    uint32_t *rec = spawn_rec(c, st, e, nb);
    // (the odd neighbour's cell: DPP quad_perm [1,0,3,2], the whole wave active)
    const int nxt = dpp_pin(__builtin_amdgcn_mov_dpp(cell, 0xb1, 0xf, 0xf, false));
    const uint32_t cw = ((uint32_t)cell & 0xffffu) | ((uint32_t)nxt << 16);
    const bool cst = ok && (lane & 1) == 0 && lane < c.S * c.L;
    uint32_t *wp = reinterpret_cast<uint32_t *>(st.env + (int64_t)e * kEnvRec + ENV_SPAWN);
    const uint32_t w1 = (spw & ~((1u << kSpawnGenShift) - 1u)) | ((uint32_t)nb << kSpawnBufShift) |
                        (ok ? SPAWN_READY : SPAWN_PARTIAL);
    if constexpr (BG) {
#pragma unroll
        for (int t = 0; t < 10; t++)
            if (64 * t + lane < kMtN) st_sc1(rec + 64 * t + lane, mt.w[t]);
        if (cst) st_sc1(rec + kSpawnCells + (lane >> 1), cw);
        if (lane == 0) st_sc1(rec + kSpawnPos, (uint32_t)mt.pos);
        __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) atomicCAS(wp, spw, w1);
    } else {
        mt_store(mt, rec, lane);
        if (cst) rec[kSpawnCells + (lane >> 1)] = cw;
        if (lane == 0) {
            rec[kSpawnPos] = (uint32_t)mt.pos;
            *wp = w1;
        }
    }
}

// The in-step spawn-ahead job of env e: one attempt from its MT state or its
// partial record, into record buffer 0.
template <int MS, int JL>
__device__ void do_spawn(const KCfg &c, const snake_state &st, int e, uint8_t *lds, int slot, int lane)
{
    WaveMT mt;
    uint32_t cellw;
    const int spw = load_reset_mt(c, st, e, mt, lane, false, cellw);
    if ((spw & 3) == SPAWN_READY) return;
    int q[MS], cell;
    bool ok = false;
    for (int a = 0; a < c.spawn_tries && !ok; a++) {   // (attempts until disjoint, at most spawn_tries)
        if (a > 0) wave_sync();
        ok = spawn_attempt<MS, JL>(c, st, mt, lds, slot, q, cell, lane);
    }
    store_spawn_record(c, st, e, mt, ok, cell, lane, (uint32_t)spw);
}

// Background spawn-ahead job (k_spawn) of env e, queued by step t's k_logic at
// generation qgen, running beside step t's resets and step t+1 (both its rules
// and its resets). Every writer of env e's MT state changes the generation with
// an atomic first or last -- k_logic's draws (atomic exchange after them), an
// auto-reset's claim (atomic add before it) -- so a job that sees another
// generation has nothing to do, and one whose inputs were being rewritten fails
// its final compare-and-swap (or is voided by the exchange landing after it).
// The record goes to buffer c.qpar, the job's queue set. Since round 5 the two
// sets' kernels run on two streams and may overlap: a job voided by k_logic's
// fruit draw (its word overwritten) may still be running when the next step's
// k_logic queues the env again into the other set, whose job then draws from
// the new state. Writing "the buffer the word does not point at" (as until
// round 5) let both jobs write the same buffer -- k_logic's exchange clears the
// buffer bit -- and a late write of the voided job could land in the published
// record. With one buffer per set the two write different buffers; jobs of one
// set run in order on one stream. A reset reads the buffer the word points at,
// and the job that published it has finished; a job continuing a partial
// record of its own set's buffer reads it whole (into registers) before it
// overwrites it.
template <int MS>
__device__ void do_spawn_bg(const KCfg &c, const snake_state &st, int e, uint32_t qgen, uint8_t *lds, int lane)
{
    uint32_t *wp = reinterpret_cast<uint32_t *>(st.env + (int64_t)e * kEnvRec + ENV_SPAWN);
    int v = 0;
    if (lane == 0) v = (int)atomicAdd(wp, 0u);   // (the memory-side value)
    uint32_t spw = (uint32_t)__shfl(v, 0);
    // (READY: nothing to do; DRAWING: another job -- an earlier step's -- has it)
    if (((spw >> kSpawnGenShift) & ((1u << kQGenBits) - 1u)) != qgen || (spw & 3u) >= SPAWN_READY) return;
    const uint32_t st0 = spw & 3u;
    {
        // mark the record as being drawn: claim_reset_mt waits for it, and a job
        // of the other queue set's kernel (they may overlap) leaves the env
        // alone. A word that moved meanwhile (a draw voided it, a reset claimed
        // it, the other job took it) ends this job.
        int won = 0;
        if (lane == 0) won = atomicCAS(wp, spw, (spw & ~3u) | SPAWN_DRAWING) == spw ? 1 : 0;
        if (!__shfl(won, 0)) return;
        spw = (spw & ~3u) | SPAWN_DRAWING;
    }
    // (fault injection for the tests, snake_debug_set "spawn_delay_ticks": the
    // job holds the record DRAWING that much longer, so resets meet it)
    if (c.spawn_delay) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned)c.spawn_delay) __builtin_amdgcn_s_sleep(32);
    }
    const int buf = (spw >> kSpawnBufShift) & (kQSets - 1);
    WaveMT mt;
    if (st0 != SPAWN_NONE) {
        const uint32_t *rec = spawn_rec(c, st, e, buf);
        mt_load_sc1(mt, rec, (int)ld_sc1(rec + kSpawnPos), lane);
    } else {
        mt_load(mt, st.mt + (int64_t)e * kMtN, st.env[(int64_t)e * kEnvRec + ENV_MTPOS], lane);
    }
    int q[MS], cell;
    bool ok = false;
    for (int a = 0; a < c.bg_tries && !ok; a++) {   // (attempts until disjoint, at most bg_tries)
        if (a > 0) wave_sync();
        ok = spawn_attempt<MS, 1>(c, st, mt, lds, 0, q, cell, lane);
    }
    store_spawn_record<true>(c, st, e, mt, ok, cell, lane, spw, c.qpar);
}

// Spawn-ahead right after an explicit reset (k_reset): the next episode's spawn
// poses drawn from the MT state the reset leaves (still in registers), up to
// kResetAheadTries permutation attempts (READY, else a PARTIAL record the step's
// workers continue). Nothing else has drawn from that state, so the record is
// exactly what the next reset would draw (spawn-ahead semantics, snake_step).
constexpr int kResetAheadTries = 4;

template <int MS, int JL>
__device__ void spawn_after_reset(const KCfg &c, const snake_state &st, int e, WaveMT &mt, uint8_t *lds,
                                  int slot, int lane)
{
    wave_sync();   // the reset's encode has read the LDS frames the draw record may overlay
    int q[MS], cell;
    bool ok = false;
    for (int a = 0; a < kResetAheadTries && !ok; a++)
        ok = spawn_attempt<MS, JL>(c, st, mt, lds, slot, q, cell, lane);
    store_spawn_record(c, st, e, mt, ok, cell, lane, (uint32_t)st.env[(int64_t)e * kEnvRec + ENV_SPAWN], 0);
}

// ---------------------------------------------------- step: the observation
// After k_logic, one launch (k_post / k_post_lean, launch_step): reset workers
// (the queued auto-resets, latency-bound, many registers, draw record in LDS,
// then the in-step spawn-ahead jobs) and the encodes of every other env's
// stacked frames (bandwidth-bound).
// The observation of env e's current frame stack (_get_obs, snake_env.py:461-472):
// the grid ring and crop centres staged in LDS, then the (staged) encode.
__device__ __forceinline__ void encode_env(const KCfg &c, const snake_state &st, const snake_out &o, int e,
                                           uint8_t *lds, int lane)
{
    const int fs = c.fs, S = c.S;
    uint8_t *frames = lds + c.lds_frames;
    int *org = reinterpret_cast<int *>(lds + c.lds_centers);
    const int cur = st.env[(int64_t)e * kEnvRec + ENV_CUR];
    stage_to_lds(frames, st.grid + (int64_t)e * c.ring_bytes, c.ring_bytes, lane);
    for (int q = lane; q < fs * S; q += kWave) {
        const int x = q / S, k = q - x * S;
        const int p = st.ctr[(int64_t)e * fs * S + q];
        org[x * kMaxSnakes + k] = pack_origin(c, p >> 8, p & 255);
    }
    wave_sync();
    encode_obs(c, frames, org, cur + 1 == fs ? 0 : cur + 1, o.obs + (int64_t)e * c.units * 8, lds, lane);
}

// RO: resets only (every-step mode, background spawn-ahead): no spawn-job path,
// fewer registers. JL: 1 the u16 draw record in LDS (KCfg.link_in_lds), 2 the
// u32 link table in LDS (KCfg.link32, batches of up to 32 768 envs), 0 the
// global link tables; one path per instantiation.
// wid = this worker (0 .. G-1): k_autoreset's block, or a block of k_post.
template <int MS, bool RO, int JL>
__device__ __forceinline__ void autoreset_worker(const int wid, const int G, uint8_t *lds)
{
    const int lane = threadIdx.x & (kWave - 1);
    const KArgs &A = kargs();
    const KCfg &c = A.c;
    const snake_state &st = A.st;
    // the shard counts of the three queues, prefix-summed: queue index j lives
    // in the shard whose [excl, incl) holds it
    const int64_t qset = kNumQ * kQShards * c.q_cap + kQCounters;
    int *qb = st.resetq + c.qpar * qset;
    int *qc = qb + kNumQ * kQShards * c.q_cap;
    const int cnt = qc[lane * kQSpread], ucnt = qc[(kQShards + lane) * kQSpread],
              ncnt = qc[(2 * kQShards + lane) * kQSpread];
    const int incl = wave_scan(cnt, lane), uincl = wave_scan(ucnt, lane), nincl = wave_scan(ncnt, lane);
    const int R = bcast(incl, kWave - 1), U = bcast(uincl, kWave - 1);
    // claim shards: min(G, kClaimShards), so that every shard has a worker
    const int nsh = min(G, kClaimShards);
    const int x = G >= kClaimShards ? (wid & (kClaimShards - 1)) : wid % nsh;
    const int P = (RO || c.bg) ? 0 : U + bcast(nincl, kWave - 1);   // (background: the spawn jobs are k_spawn's)
    const int T = R + P;
    if (wid == 0 && lane == 0 && R > 0) {
        atomicAdd(&g_resets_run, (unsigned long long)R);
        if (c.diag) atomicAdd(&g_resets_timed, (unsigned long long)R);
    }
    // env of job j of queue q
    // (only the inclusive prefix sums stay live across the jobs: the shard of
    // job j is the number of shards whose prefix ends at or before j)
    auto job_env = [&](int q, int j, int qincl) {
        const int sh = __popcll(__ballot(qincl <= j));
        const int base = sh ? bcast(qincl, sh - 1) : 0;
        return qb[(q * kQShards + sh) * c.q_cap + j - base];
    };
    // job idx < R: the step's resets (high priority, the critical path); then
    // the urgent spawn-ahead jobs, then the others. A worker's first job is its
    // block index, the next ones are claimed once it is free (a slow reset
    // never holds up a job another worker could take): worker w claims on
    // shard x = w % kClaimShards, whose n-th claim is job G + x + kClaimShards * n.
    int idx = wid, nx = 0;
    for (;;) {
        // (the arguments afresh for each job: nothing of them stays live across
        // jobs; so is the lane index, or every lane mask derived from it -- the
        // MT word bounds, the scan steps -- would be held, spilled, for the whole
        // kernel instead of recomputed by one compare)
        const KArgs &J = kargs();
        int lane = threadIdx.x & (kWave - 1);
        __asm__ volatile("" : "+v"(lane));
        if (idx < R) {
            __builtin_amdgcn_s_setprio(3);
            const int e = job_env(0, idx, incl);
#ifdef SNAKE_FUSE_DEBUG
            if ((e < 0 || e >= J.c.N) && FDBG_BAD(1, e)) { idx = 1 << 30; break; }
#endif
            ITEM_T0();
            WaveMT mt;
            uint32_t cellw;
            const int spst = J.c.bg ? claim_reset_mt(J.c, J.st, e, mt, lane, cellw)
                                    : load_reset_mt(J.c, J.st, e, mt, lane, true, cellw);
            if (J.c.diag && lane == 0 && (spst & 3) == SPAWN_READY) DIAG_ADD(g_spawn_hits);
            if (J.c.diag && lane == 0 && (spst & 3) == SPAWN_PARTIAL) DIAG_ADD(g_reset_part);
            do_reset<MS, JL>(J.c, J.st, J.o, e, mt, lds, wid, spst, cellw, lane);
            ITEM_LOG(wid, 2 - (spst & 3), e);
        } else if (!RO && idx < R + P) {
            if (J.c.spawn_prio == 0) __builtin_amdgcn_s_setprio(0);   // (s_setprio takes an immediate)
            else if (J.c.spawn_prio == 1) __builtin_amdgcn_s_setprio(1);
            else if (J.c.spawn_prio == 2) __builtin_amdgcn_s_setprio(2);
            else __builtin_amdgcn_s_setprio(3);
            const int j = idx - R;
            const int e = j < U ? job_env(1, j, uincl) : job_env(2, j - U, nincl);
#ifdef SNAKE_FUSE_DEBUG
            if ((e < 0 || e >= J.c.N) && FDBG_BAD(2, e)) { idx = 1 << 30; break; }
#endif
            if (J.c.diag && lane == 0) DIAG_ADD(g_spawn_jobs);
            ITEM_T0();
            do_spawn<MS, JL>(J.c, J.st, e, lds, wid, lane);
            ITEM_LOG(wid, j < U ? 3 : 4, e);
        }
        int v = 0;
        if (lane == 0) v = atomicAdd(&qc[(kQClaim + x) * kQSpread], 1);
        nx = bcast(v, 0);
        idx = G + x + nsh * nx;
        if (idx >= T) break;
    }
    // Every worker ends with exactly one failing claim, so the shard's claims
    // number its jobs + its workers, and the worker whose failing claim is the
    // shard's last finishes the shard. The last shard to finish re-zeroes the
    // step's counters for the next step: every worker has read its counts and
    // made its last claim by then (no host-side step parity, one extra atomic
    // per shard).
    const int jobs_x = T > G + x ? (nsh == kClaimShards ? (T - G - x + kClaimShards - 1) / kClaimShards
                                                       : (T - G - x + nsh - 1) / nsh) : 0;
    const int workers_x = nsh == kClaimShards ? (G - x + kClaimShards - 1) / kClaimShards : (G - x + nsh - 1) / nsh;
    if (nx == jobs_x + workers_x - 1) {
        int d = 0;
        if (lane == 0) d = atomicAdd(&qc[kQDone * kQSpread], 1);
        if (bcast(d, 0) == nsh - 1)   // (background: the reset counters only)
            for (int q = lane; q < kQSpGen; q += kWave)
                if (!c.bg || q < kQShards || (q >= kQClaim && q <= kQDone)) qc[q * kQSpread] = 0;
    }
}

template <int MS, bool RO, int JL>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kResetWavesPerEU))) k_autoreset(const KArgs)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    autoreset_worker<MS, RO, JL>((int)blockIdx.x, (int)gridDim.x, lds);
}

// Background spawn-ahead (KCfg.bg): the step's spawn-ahead jobs, run by
// spawn_slots one-wave workers on a stream of their own that no step waits for
// except the one two steps later, whose k_logic refills this queue set
// (launch_step); do_spawn_bg says how they stay out of the resets' way. Jobs
// are claimed on 16 claim shards like k_autoreset's, whose last worker
// re-zeroes the set's spawn counters.
template <int MS>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kResetWavesPerEU))) k_spawn(const KArgs)
{
    const KArgs &A = kargs();
    const KCfg &c = A.c;
    const snake_state &st = A.st;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int lane = threadIdx.x;
    if (c.spawn_prio == 0) __builtin_amdgcn_s_setprio(0);
    else if (c.spawn_prio == 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(2);
    int *qb = st.resetq + (int64_t)c.qpar * (kNumQ * kQShards * c.q_cap + kQCounters);
    int *qc = qb + kNumQ * kQShards * c.q_cap;
    const int ucnt = qc[(kQShards + lane) * kQSpread], ncnt = qc[(2 * kQShards + lane) * kQSpread];
    const int uincl = wave_scan(ucnt, lane), nincl = wave_scan(ncnt, lane);
    const int U = bcast(uincl, kWave - 1), T = U + bcast(nincl, kWave - 1);
    const int G = (int)gridDim.x, nsh = min(G, kClaimShards);
    const int x = G >= kClaimShards ? (int)(blockIdx.x & (kClaimShards - 1)) : (int)blockIdx.x % nsh;
    auto job_env = [&](int q, int j, int qincl) {
        const int sh = __popcll(__ballot(qincl <= j));
        const int base = sh ? bcast(qincl, sh - 1) : 0;
        return qb[(q * kQShards + sh) * c.q_cap + j - base];
    };
    int nx = -1;   // (a worker with no first job makes one failing claim below)
    int idx = blockIdx.x;
    if (idx >= T) {
        int v = 0;
        if (lane == 0) v = atomicAdd(&qc[(kQSpClaim + x) * kQSpread], 1);
        nx = bcast(v, 0);
    }
    for (; idx < T;) {
        const int ent = idx < U ? job_env(1, idx, uincl) : job_env(2, idx - U, nincl);
        const int e = ent & ((1 << (32 - kQGenBits)) - 1);
        const uint32_t qgen = (uint32_t)ent >> (32 - kQGenBits);
        if (c.diag && lane == 0) DIAG_ADD(g_spawn_jobs);
        const KArgs &J = kargs();
        do_spawn_bg<MS>(J.c, J.st, e, qgen, lds, lane);
        int v = 0;
        if (lane == 0) v = atomicAdd(&qc[(kQSpClaim + x) * kQSpread], 1);
        nx = bcast(v, 0);
        idx = G + x + nsh * nx;
    }
    // the shard's last claim finishes the shard; the last shard re-zeroes (as in
    // k_autoreset, with this kernel's claim and done counters)
    const int jobs_x = T > G + x ? (T - G - x + nsh - 1) / nsh : 0;
    const int workers_x = (G - x + nsh - 1) / nsh;
    if (nx == jobs_x + workers_x - 1) {
        int d = 0;
        if (lane == 0) d = atomicAdd(&qc[kQSpDone * kQSpread], 1);
        if (bcast(d, 0) == nsh - 1) {
            // write-through zeroes, drained, then the set's finished count: a
            // k_logic that reads the count (sc1) then adds to these counters
            // from any XCD (MI355X_MICROARCH.md, inter-workgroup hand-off)
            for (int q = kQShards + lane; q < kNumQ * kQShards; q += kWave)
                st_sc1(reinterpret_cast<uint32_t *>(&qc[q * kQSpread]), 0u);
            if (lane <= kClaimShards) st_sc1(reinterpret_cast<uint32_t *>(&qc[(kQSpClaim + lane) * kQSpread]), 0u);   // (claims + done)
            __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0) atomicAdd(reinterpret_cast<unsigned *>(&qc[kQSpGen * kQSpread]), 1u);
        }
    }
}

__device__ __forceinline__ void encode_one(const KCfg &c, const snake_state &st, const snake_out &o, const int e)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int lane = threadIdx.x;
    // a reset env's obs is written by its reset; in every-step mode only the
    // envs rejected for an invalid action (left unchanged) are not reset
    if (c.autoreset == 2 ? o.err[e] != 1 : (c.autoreset && o.ep_done[e])) return;
    if (c.encode_prio == 1) __builtin_amdgcn_s_setprio(1);      // (setprio takes an immediate)
    else if (c.encode_prio == 2) __builtin_amdgcn_s_setprio(2);
    else if (c.encode_prio == 3) __builtin_amdgcn_s_setprio(3);
    encode_env(c, st, o, e, lds, lane);
}

__global__ void __launch_bounds__(64) k_encode(const KCfg c, const snake_state st, const snake_out o)
{
    encode_one(c, st, o, (int)blockIdx.x);
}

// k_encode over c.enc_per_wave consecutive envs per wave: the next env's grid
// ring, current slot, crop centres and reset flag are loaded into registers
// before this env's encode, so their memory round trip overlaps it (a
// one-env wave waits for its ring with nothing else to do; the encode is
// latency- and occupancy-bound beside the reset workers). NPF = 16-byte ring
// chunks per lane kept in flight (ring_bytes <= NPF * 1024).
template <int NPF>
__device__ __forceinline__ void encode_multi(const KCfg &c, const snake_state &st, const snake_out &o, const int b)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int lane = threadIdx.x;
    if (c.encode_prio == 1) __builtin_amdgcn_s_setprio(1);
    else if (c.encode_prio == 2) __builtin_amdgcn_s_setprio(2);
    else if (c.encode_prio == 3) __builtin_amdgcn_s_setprio(3);
    const int fs = c.fs, S = c.S, n16 = c.ring_bytes >> 4, fsS = fs * S;
    uint8_t *frames = lds + c.lds_frames;
    int *org = reinterpret_cast<int *>(lds + c.lds_centers);
    const int e_begin = b * c.enc_per_wave, e_end = min(c.N, e_begin + c.enc_per_wave);
    // (one vector value, not an array: an array of uint4 carried across the
    // loop was demoted to scratch)
    typedef uint32_t pf_t __attribute__((ext_vector_type(4 * NPF)));
    pf_t pf = {};
    int pcur = 0, pctr = 0, pskip = 0;
#define SNAKE_ENC_FETCH(EE)                                                                        \
    do {                                                                                           \
        const int64_t e_ = (EE);                                                                   \
        const uint4 *src_ = reinterpret_cast<const uint4 *>(st.grid + e_ * c.ring_bytes);          \
        _Pragma("unroll") for (int u = 0; u < NPF; u++) {   /* (clamped: no per-chunk branch) */   \
            const uint4 x_ = src_[min(lane + u * kWave, n16 - 1)];                                 \
            pf[4 * u] = x_.x; pf[4 * u + 1] = x_.y; pf[4 * u + 2] = x_.z; pf[4 * u + 3] = x_.w;     \
        }                                                                                          \
        pcur = st.env[e_ * kEnvRec + ENV_CUR];                                                     \
        pctr = lane < fsS ? st.ctr[e_ * fsS + lane] : 0;                                           \
        pskip = c.autoreset ? o.ep_done[e_] : 0;                                                   \
    } while (0)
    if (e_begin < e_end) SNAKE_ENC_FETCH(e_begin);
    for (int e = e_begin; e < e_end; e++) {
        const int cur = pcur, skip = pskip;   // (its reset writes the obs of a reset env)
        if (!skip) {
            uint4 *d4 = reinterpret_cast<uint4 *>(frames);
#pragma unroll
            for (int u = 0; u < NPF; u++)
                d4[min(lane + u * kWave, n16 - 1)] = make_uint4(pf[4 * u], pf[4 * u + 1], pf[4 * u + 2], pf[4 * u + 3]);
            if (lane < fsS) {
                const int x = lane / S, k = lane - x * S;
                org[x * kMaxSnakes + k] = pack_origin(c, pctr >> 8, pctr & 255);
            }
        }
        if (e + 1 < e_end) SNAKE_ENC_FETCH(e + 1);   // in flight during this env's encode
        if (!skip) {
            wave_sync();
            encode_obs(c, frames, org, cur + 1 == fs ? 0 : cur + 1, o.obs + (int64_t)e * c.units * 8, lds, lane);
            wave_sync();   // the LDS frames are rewritten for the next env
        }
    }
#undef SNAKE_ENC_FETCH
}

// The shared phase as one launch: blocks [0, reset_slots) are the reset workers
// (autoreset_worker), the rest the encodes (NPF = 0: one env per block,
// encode_one; else encode_multi<NPF>). Dispatched in block order, so the workers
// go first; one launch instead of a fork onto a side stream and a join (round 3:
// cfg3 0.0970 -> 0.0941 ms, cfg2 0.0591 -> 0.0539); the kernel's registers and
// LDS are the larger of the two. JL: the workers' draw record (1) or u32 link
// table (2) in LDS, else their global link tables (boards of more than 18 368
// spawn poses).
// ---------------------------------------------------------- table encode
// The observation of c.enc_per_wave consecutive envs per wave (_encode
// snake_env.py:474-519 + the frame stack :444-472) as table lookups. Per 8-byte
// unit (snake k, window row i, column j, frame f: obs (S, oh, ow, 8 fs)) the grid
// byte v of frame f at that window cell comes from a zero-bordered LDS image of
// the env's frames (no bounds test: cells outside the grid read 0), and the
// unit's 8 one-hot channels are the table entry pat[k][v] (onehot()). A lane's
// units are the same for every env: their descriptors desc[u] = (i * pw + j) |
// (f * 16 + k) << 16 are built once per wave, and per env only the window
// origins base[f * 16 + k] = (LDS byte of the window origin in frame f, byte
// offset of pat[k]) change. Per 16-byte store: one descriptor pair, two window
// origins, two grid bytes and two patterns from LDS, four address adds. The
// next env's frames (NPW dwords per lane), slot, crop centres and reset flag
// are loaded into registers during this env's encode (as encode_lean_block).
constexpr int kPatV = 160;   // grid byte values 10 * id + code (id < 16, code <= 5)

template <int T>
__device__ __forceinline__ void tsync()
{
    if constexpr (T == kWave) wave_sync();
    else __syncthreads();
}

// FU (k_step): the frames and the hand-off record (slot, reset flag, crop
// centres) of the logic wave that finished these envs in this launch, all read
// with write-through-coherent (sc1) loads after its done flag
template <int NPW, int T = kWave, bool FU = false>
__device__ void encode_tbl_block(const KCfg &c, const snake_state &st, const snake_out &o, const int blk)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int lane = threadIdx.x;
    if (c.encode_prio == 1) __builtin_amdgcn_s_setprio(1);
    else if (c.encode_prio == 2) __builtin_amdgcn_s_setprio(2);
    else if (c.encode_prio == 3) __builtin_amdgcn_s_setprio(3);
    uint8_t *pf = lds;                                                   // fs * pframe bytes
    uint2 *base = reinterpret_cast<uint2 *>(lds + c.tbl_base);           // [fs][16]
    uint8_t *pat = lds + c.tbl_pat;                                      // uint2 [S][kPatV]
    uint32_t *desc = reinterpret_cast<uint32_t *>(lds + c.tbl_desc);     // [units]
    const int S = c.S, fs = c.fs, fsS = fs * S;
    const int wpr = c.W >> 2, nw = c.H * wpr, nwt = fs * nw, gsw = c.grid_stride >> 2;
    // per prefetched dword: ring word index and LDS dword index (clamped: the
    // lanes past the end repeat the last word, same source, same destination)
    int src[NPW], dst[NPW];
#pragma unroll
    for (int u = 0; u < NPW; u++) {
        const int x = min(lane + u * T, nwt - 1);
        const int s = x / nw, xx = x - s * nw;
        const int r = fdiv((uint32_t)xx, c.mag_wpr, wpr), c4 = xx - r * wpr;
        src[u] = s * gsw + xx;
        dst[u] = (s * c.pframe + (r + c.vr) * c.pw + c.lp) / 4 + c4;
    }
    // once per wave: the zero image, the patterns of the codes that occur (0, 1,
    // 2 and 10 * id + 3..5 for id < S), the unit descriptors
    zero_lean<T>(c, pf, lane);
    const int npv = 3 + 3 * S;   // occurring codes per snake
    for (int x = lane; x < S * npv; x += T) {
        const int k = x / npv, r = x - k * npv;
        const int v = r < 3 ? r : 10 * ((r - 3) / 3) + 3 + (r - 3) % 3;
        const unsigned long long b = onehot(v, k);
        reinterpret_cast<uint2 *>(pat)[k * kPatV + v] = make_uint2((uint32_t)b, (uint32_t)(b >> 32));
    }
    for (int u = lane; u < c.units; u += T) {
        const int kk = (int)__umulhi((uint32_t)u, c.mag_ups), r0 = u - kk * c.ups;
        const int ii = (int)__umulhi((uint32_t)r0, c.mag_rowl), r1 = r0 - ii * c.rowl;
        const int jj = fdiv((uint32_t)r1, c.mag_fs, fs), ff = r1 - jj * fs;
        desc[u] = (uint32_t)(ii * c.pw + jj) | ((uint32_t)(ff * kMaxSnakes + kk) << 16);
    }
    const int e_begin = blk * c.enc_per_wave, e_end = min(c.N, e_begin + c.enc_per_wave);
    uint32_t w[NPW];
    int pcur = 0, pctr = 0, pskip = 0;
#define SNAKE_TBL_FETCH(EE)                                                                        \
    do {                                                                                           \
        const int64_t e_ = (EE);                                                                   \
        const uint32_t *r32_ = reinterpret_cast<const uint32_t *>(st.grid + e_ * c.ring_bytes);    \
        if constexpr (FU) {                                                                        \
            _Pragma("unroll") for (int u = 0; u < NPW; u++) w[u] = ld_sc1(r32_ + src[u]);          \
            const uint4 h_ = ld_sc1_128(st.resetq + c.fu_hoff + 4 * e_);                           \
            pcur = (int)(h_.x & 255u);                                                             \
            pskip = (int)((h_.x >> 8) & 1u);                                                       \
            pctr = lane < fsS ? (int)(((lane < 2 ? h_.y : h_.z) >> (16 * (lane & 1))) & 0xffffu) : 0; \
        } else {                                                                                   \
            _Pragma("unroll") for (int u = 0; u < NPW; u++) w[u] = r32_[src[u]];                   \
            pcur = st.env[e_ * kEnvRec + ENV_CUR];                                                 \
            pctr = lane < fsS ? st.ctr[e_ * fsS + lane] : 0;                                       \
            pskip = c.autoreset ? o.ep_done[e_] : 0;                                               \
        }                                                                                          \
    } while (0)
    if (e_begin < e_end) SNAKE_TBL_FETCH(e_begin);
    const int chunks = c.units >> 1;
    // a lane's chunks all in one pass (cfg3: 242 chunks): their descriptors in
    // registers for every env of the wave, one LDS level less per lookup chain
    const bool one = T == kWave && chunks <= 4 * T;
    uint2 dr[4];
    if constexpr (T == kWave) if (one) {
        tsync<T>();
#pragma unroll
        for (int t = 0; t < 4; t++) dr[t] = reinterpret_cast<const uint2 *>(desc)[min(t * T + lane, chunks - 1)];
    }
    for (int e = e_begin; e < e_end; e++) {
        const int cur = pcur, skip = pskip;   // (a reset env's obs is written by its reset)
        tsync<T>();                          // (the previous encode has read the LDS image)
        if (!skip) {
#pragma unroll
            for (int u = 0; u < NPW; u++) reinterpret_cast<uint32_t *>(pf)[dst[u]] = w[u];
            if (lane < fsS) {
                // ring slot s = lane / S holds frame f = s - (the oldest slot), mod fs
                const int s = lane / S, k = lane - s * S, slot0 = cur + 1 == fs ? 0 : cur + 1;
                const int f = s >= slot0 ? s - slot0 : s - slot0 + fs;
                const uint32_t gb = (uint32_t)(s * c.pframe) +
                                    (c.vr ? (uint32_t)((pctr >> 8) * c.pw + (pctr & 255) + c.lp - c.vr) : 0u);
                base[f * kMaxSnakes + k] = make_uint2(gb, (uint32_t)(k * kPatV * 8));
            }
        }
        if (e + 1 < e_end) SNAKE_TBL_FETCH(e + 1);   // in flight during this env's encode
        if (!skip) {
            tsync<T>();
            const auto rs = __builtin_amdgcn_make_buffer_rsrc(o.obs + (int64_t)e * c.units * 8, 0, c.units * 8, 0x00020000);
            auto lookup = [&](uint2 dd) {   // units 2q, 2q + 1 of descriptor pair dd
                const uint2 b0 = base[dd.x >> 16], b1 = base[dd.y >> 16];
                const uint32_t v0 = pf[b0.x + (dd.x & 0xffffu)], v1 = pf[b1.x + (dd.y & 0xffffu)];
                const uint2 p0 = *reinterpret_cast<const uint2 *>(pat + b0.y + 8 * v0);
                const uint2 p1 = *reinterpret_cast<const uint2 *>(pat + b1.y + 8 * v1);
                return (v4u){p0.x, p0.y, p1.x, p1.y};
            };
            if (T == kWave && one) {
                v4u r[4];
#pragma unroll
                for (int t = 0; t < 4; t++) r[t] = lookup(dr[t]);
#pragma unroll
                for (int t = 0; t < 4; t++)
                    if (t * T + lane < chunks) obs_store_rs(rs, 16 * (t * T + lane), r[t]);
            } else {
            // CP chunks per lane and pass, their lookup chains interleaved
            // (clamped reads; only the chunks that exist are stored); two in
            // four-wave workgroups (register budget)
            constexpr int CP = T == kWave ? 4 : 2;
            for (int q0 = 0; q0 < chunks; q0 += CP * T) {
                v4u r[CP];
#pragma unroll
                for (int t = 0; t < CP; t++)
                    r[t] = lookup(reinterpret_cast<const uint2 *>(desc)[min(q0 + t * T + lane, chunks - 1)]);
#pragma unroll
                for (int t = 0; t < CP; t++)
                    if (q0 + t * T + lane < chunks) obs_store_rs(rs, 16 * (q0 + t * T + lane), r[t]);
            }
            }
        }
    }
#undef SNAKE_TBL_FETCH
}

// ------------------------------------------------------------ fused step
// k_step (round 6): the whole step as ONE launch on boards whose encodes take
// the table form in one wave and whose hand-off record holds the crop centres
// (one frame, S <= 4: cfg2, cfg3, cfg4), no background spawn kernel. Blocks
// [0, nlg) are k_logic's env groups, the next reset_slots blocks the reset
// workers, the rest the table encodes (4 envs each). The encodes of a group
// start as soon as that group's rules are done instead of after the last
// group and a kernel boundary, so k_logic's latency chain runs beside the
// encodes' stores.
// Dispatch order, timing and placement are not assumed (MI355X_MICROARCH.md
// "Workgroup dispatch", contract [G]): every logic group is CLAIMED (an atomic
// exchange of the step's epoch) by whichever wave gets it first -- its own
// block, or an encode block of that group that finds it unclaimed, or a reset
// worker that has waited long -- and the claimer runs it at once without
// waiting on anything. A wave waits only for a group that is claimed, i.e.
// running, so the launch cannot deadlock.
// Hand-offs (R1 of the guide's visibility rules): the logic wave's stores that
// another wave of the launch reads or writes are write-through (sc1) stores --
// the new frame, the env record, the queue entries, the spawn status word, a
// rewritten MT key, the encodes' hand-off record -- drained (vmcnt(0)) before
// the group's done flag (sc1 store of the epoch) and its logic-done count (an
// atomic add on shard blk % 64); an env whose episode ended stores nothing its
// auto-reset rewrites. The encodes poll the flag and read their inputs with sc1
// loads only; the workers poll the 64 counts, then one agent-scope acquire,
// then the queues and env state as before. Epochs: the library's per-state step
// count (launch_step); the counts grow by their shard's group count per step.
// Every wait is bounded (kFuseWait): past it the wave carries on and the launch
// counts the timeout ("fused_timeout"), the results are then undefined.
__device__ unsigned long long g_fused_timeout[kDiagSlots * kDiagSpread];
constexpr unsigned long long kFuseWait = 10000000ull;   // 100 ms of the 100 MHz clock
constexpr unsigned long long kFuseHelp = 2000ull;       // 20 us: a waiting worker then claims unclaimed groups

// (Everything here is inlined into k_step: kargs() reads the kernarg segment
// pointer, which a called function does not have -- an out-of-line
// fused_logic read its KCfg from garbage and faulted, round 6.)
__device__ __forceinline__ bool fused_claim(const int g)
{
    const KCfg &c = kargs().c;
    uint32_t *claim = reinterpret_cast<uint32_t *>(kargs().st.resetq + c.fu_claim) + g;
    int won = 0;
    if ((threadIdx.x & (kWave - 1)) == 0) won = atomicExch(claim, c.epoch) != c.epoch ? 1 : 0;
    return __shfl(won, 0) != 0;
}

__device__ __forceinline__ bool fused_group_done(const int g)
{
    const KCfg &c = kargs().c;
    const uint32_t *done = reinterpret_cast<const uint32_t *>(kargs().st.resetq + c.fu_done) + g;
    return (uint32_t)__shfl((int)ld_sc1(done), 0) == c.epoch;
}

// an encode block's wait for its group's rules, which some wave has claimed
__device__ __forceinline__ void fused_wait_group(const int g)
{
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (!fused_group_done(g)) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > kFuseWait) {
            if ((threadIdx.x & (kWave - 1)) == 0) DIAG_ADD(g_fused_timeout);
            return;
        }
        __builtin_amdgcn_s_sleep(4);
    }
}

// A reset worker's wait for every group's rules (the queues complete): -1 once
// they are done (or the wait timed out), else a group it has just claimed and
// must run -- once it has waited kFuseHelp, every group still unclaimed, from a
// worker-specific start (`scan`: the next scan position, -1 before the first)
__device__ __forceinline__ int fused_wait_all(const int wid, const unsigned long long t0, int &scan)
{
    const int lane = threadIdx.x & (kWave - 1);
    for (;;) {
        const KCfg &c = kargs().c;
        const int nlg = c.nlg;
        // shard s (lane s) counts the groups g = s mod 64: (nlg - s + 63) / 64 of them per step
        const uint32_t ns = lane < nlg ? (uint32_t)((nlg - lane + kQShards - 1) / kQShards) : 0u;
        const uint32_t v = ld_sc1(reinterpret_cast<const uint32_t *>(kargs().st.resetq + c.fu_ldone) + lane * kQSpread);
        if (__ballot(v != c.epoch * ns) == 0ull) return -1;
        const unsigned long long dt = __builtin_amdgcn_s_memrealtime() - t0;
        if (dt > kFuseWait) {
            if (lane == 0) DIAG_ADD(g_fused_timeout);
            return -1;
        }
        if (dt > kFuseHelp && scan < nlg) {
            if (scan < 0) scan = 0;
            for (; scan < nlg; scan += kWave) {
                const int g = (wid * 61 + scan + lane) % nlg;
                const KCfg &c2 = kargs().c;
                const uint32_t cl = scan + lane < nlg ? ld_sc1(reinterpret_cast<const uint32_t *>(kargs().st.resetq + c2.fu_claim) + g)
                                                      : c2.epoch;
                unsigned long long m = __ballot(cl != c2.epoch);
                while (m) {
                    const int L = __ffsll((long long)m) - 1;
                    m &= m - 1;
                    const int gg = __shfl(g, L);
                    if (fused_claim(gg)) return gg;   // (the next call rescans this pass)
                }
            }
        }
        __builtin_amdgcn_s_sleep(8);
    }
}

// (four waves per SIMD: at most 128 VGPRs; the rules alone take 100, the
// worker path in k_post 71)
template <int MS, int NPW, int JL>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) k_step(const KArgs)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    PTIME(0);
    const int b = (int)blockIdx.x;
    const int nlg = kargs().c.nlg, G = kargs().c.reset_slots;
    const int roles = kargs().c.fu_roles;   // (snake_debug_set "fuse_roles": 7 = all)
    const int role = b < nlg ? 0 : (b < nlg + G ? 1 : 2);   // rules, reset worker, encodes
    if (!(roles & (1 << role))) return;
    const int j = b - nlg - G;   // (encodes: envs 4j .. 4j + 3, all of logic group 4j / (64 / MS))
    const int eg = (4 * j) / (kWave / MS);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    int scan = -1;
    // the rules of every group this wave claims, at ONE inlined site
    for (int it = 0;; it++) {
        int grp = -1;
        if (role == 0) {
            if (it == 0 && fused_claim(b)) grp = b;
        } else if (role == 2) {
            if (it == 0 && !fused_group_done(eg) && fused_claim(eg)) grp = eg;
        } else {
            grp = fused_wait_all(b - nlg, t0, scan);
        }
        if (grp < 0) break;
        LogicIn in;
        logic_load<MS, false>(grp, in);
        logic_body<MS, false, true>(grp, in);
        FDBG_MARK(3);
    }
    if (role == 0) { PTIME(1); return; }
    if (role == 1) {
        // the queues, env records, MT keys and spawn records the groups published
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
        FDBG_MARK(4);
        autoreset_worker<4, false, JL>(b - nlg, G, lds);
        FDBG_MARK(5);
        PTIME(1);
        return;
    }
    if (4 * j >= kargs().c.N && FDBG_BAD(6, j)) return;
    fused_wait_group(eg);
    FDBG_MARK(7);
    const KArgs &A = kargs();
    encode_tbl_block<NPW, kWave, true>(A.c, A.st, A.o, j);
    PTIME(1);
}

// NPF > 0: encode_multi<NPF>; 0: encode_one; -NPW: encode_tbl_block<NPW>
template <int MS, int NPF, bool RO, int JL>
__global__ void __launch_bounds__(64) k_post(const KArgs)
{
    PTIME(0);
    const int G = kargs().c.reset_slots, b = (int)blockIdx.x;
    if (b < G) {
        extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
#ifdef SNAKE_DIAG_ENC2   // (diagnostic: the second, encode-only launch, see launch_step)
        if (kargs().aux) return;
#endif
        autoreset_worker<MS, RO, JL>(b, G, lds);
    } else {
#ifdef SNAKE_DIAG_NO_ENCODE   // (diagnostic build: instruction counts without the encodes)
        return;
#endif
        const KArgs &A = kargs();
        if constexpr (NPF == 0) encode_one(A.c, A.st, A.o, b - G);
        else if constexpr (NPF < 0) encode_tbl_block<-NPF>(A.c, A.st, A.o, b - G);
        else encode_multi<NPF>(A.c, A.st, A.o, b - G);
    }
    PTIME(1);
}

// Lean encode over c.enc_per_wave consecutive envs per workgroup of T = 256
// threads (W % 4 == 0, rings of 513 to 2 048 dwords: cfg5's 40x40 x 4 frames):
// the next env's frames (NPW dwords per thread), current slot, crop centres and
// reset flag are loaded into registers while this env is encoded, one memory
// round trip per env in the shadow of the previous encode; the zero border of
// the LDS image is written once per workgroup. The LDS destination of every
// prefetched dword is the same for every env (computed once). Four waves share
// one LDS image (cfg5 k_encode 91 -> 66 us against one wave per env, round 3).
template <int NPW, int T>
__device__ __forceinline__ void encode_lean_block(const KCfg &c, const snake_state &st, const snake_out &o,
                                                  const int blk)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int lane = threadIdx.x;
    if (c.encode_prio == 1) __builtin_amdgcn_s_setprio(1);
    else if (c.encode_prio == 2) __builtin_amdgcn_s_setprio(2);
    else if (c.encode_prio == 3) __builtin_amdgcn_s_setprio(3);
    uint8_t *pf = lds;
    int *base = reinterpret_cast<int *>(lds + c.fs * c.pframe);
    uint32_t *p32 = reinterpret_cast<uint32_t *>(pf);
    const int wpr = c.W >> 2, nw = c.H * wpr, nwt = c.fs * nw, gsw = c.grid_stride >> 2, fsS = c.fs * c.S;
    auto sync = [&]() {
        if constexpr (T == kWave) wave_sync();
        else __syncthreads();
    };
    // per prefetched dword: ring word index and LDS dword index (clamped: the
    // threads past the end repeat the last word, same source, same destination)
    int src[NPW], dst[NPW];
#pragma unroll
    for (int u = 0; u < NPW; u++) {
        const int x = min(lane + u * T, nwt - 1);
        const int s = x / nw, xx = x - s * nw;
        const int r = fdiv((uint32_t)xx, c.mag_wpr, wpr), c4 = xx - r * wpr;
        src[u] = s * gsw + xx;
        dst[u] = (s * c.pframe + (r + c.vr) * c.pw + c.lp) / 4 + c4;
    }
    zero_lean<T>(c, pf, lane);
    const int e_begin = blk * c.enc_per_wave, e_end = min(c.N, e_begin + c.enc_per_wave);
    uint32_t w[NPW];
    int pcur = 0, pctr = 0, pskip = 0;
#define SNAKE_LEAN_FETCH(EE)                                                                       \
    do {                                                                                           \
        const int64_t e_ = (EE);                                                                   \
        const uint32_t *r32_ = reinterpret_cast<const uint32_t *>(st.grid + e_ * c.ring_bytes);    \
        _Pragma("unroll") for (int u = 0; u < NPW; u++) w[u] = r32_[src[u]];                       \
        pcur = st.env[e_ * kEnvRec + ENV_CUR];                                                     \
        pctr = lane < fsS ? st.ctr[e_ * fsS + lane] : 0;                                           \
        pskip = c.autoreset ? o.ep_done[e_] : 0;                                                   \
    } while (0)
    if (e_begin < e_end) SNAKE_LEAN_FETCH(e_begin);
    for (int e = e_begin; e < e_end; e++) {
        const int cur = pcur, skip = pskip;   // (a reset env's obs is written by its reset)
        sync();                               // (the previous encode has read the LDS image)
        if (!skip) {
#pragma unroll
            for (int u = 0; u < NPW; u++) p32[dst[u]] = w[u];
            if (lane < fsS) {
                const int x = lane / c.S, k = lane - x * c.S;
                base[x * kMaxSnakes + k] = c.vr ? (pctr >> 8) * c.pw + (pctr & 255) + c.lp - c.vr : 0;
            }
        }
        if (e + 1 < e_end) SNAKE_LEAN_FETCH(e + 1);   // in flight during this env's encode
        if (!skip) {
            sync();
            encode_lean<T>(c, pf, base, cur + 1 == c.fs ? 0 : cur + 1, o.obs + (int64_t)e * c.units * 8, lane);
        }
    }
#undef SNAKE_LEAN_FETCH
}

// The shared phase of a board with four-wave lean encodes (cfg5) as one launch:
// workgroups [0, ceil(reset_slots / 4)) hold four independent workers each
// (wave w of workgroup b is worker 4b + w, with its own KCfg.lds_worker bytes of
// LDS -- frames, centres, fruit buffer, no draw record -- and its own global
// link table for the attempts it runs: no workgroup barrier on their path), the
// rest are lean-encode workgroups. RO: background spawn-ahead (the default on
// these boards), the workers run the resets only; else also the in-step
// spawn-ahead attempts. One launch instead of the fork/join of round 2 (12 and
// 16 us of cross-stream latency per step at cfg5).
template <int MS, bool RO, bool TBL>
__global__ void __launch_bounds__(256) k_post_lean(const KArgs)
{
    PTIME(0);
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int G = kargs().c.reset_slots, GB = (G + 3) >> 2, b = (int)blockIdx.x;
    if (b < GB) {
        const int wave = (int)(threadIdx.x >> 6), wid = 4 * b + wave;
        if (wid < G) autoreset_worker<MS, RO, 0>(wid, G, lds + wave * kargs().c.lds_worker);
    } else {
        const KArgs &A = kargs();
        if constexpr (TBL) encode_tbl_block<8, 256>(A.c, A.st, A.o, b - GB);
        else encode_lean_block<8, 256>(A.c, A.st, A.o, b - GB);
    }
    PTIME(1);
}

template <int MS, int JL>
__global__ void __launch_bounds__(64) k_reset(const KArgs)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int lane = threadIdx.x;
    // one env per block with the link table in LDS (JL), else reset_slots
    // workers striding over the envs, each with its own global link table
    for (int e = blockIdx.x; e < kargs().c.N; e += gridDim.x) {
        const KArgs &J = kargs();
        const uint8_t *mask = (const uint8_t *)J.aux;
        if (mask && !mask[e]) continue;
        WaveMT mt;
        uint32_t cellw;
        const int spst = load_reset_mt(J.c, J.st, e, mt, lane, true, cellw);
        do_reset<MS, JL>(J.c, J.st, J.o, e, mt, lds, blockIdx.x, spst, cellw, lane);
        // with spawn-ahead on, the next reset's poses are drawn now, off the step
        const KArgs &J2 = kargs();
        if (J2.c.spawn_thr >= 0) spawn_after_reset<MS, JL>(J2.c, J2.st, e, mt, lds, blockIdx.x, lane);
    }
}

// np.random.seed(s): mt19937_seed (init_genrand), pos = 624.
__global__ void k_seed(const KCfg c, const snake_state st, uint32_t base, long long off)
{
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= c.N) return;
    uint32_t s = base + (uint32_t)(off + e);
    uint32_t *g = st.mt + (int64_t)e * kMtN;
    for (int pos = 0; pos < kMtN; pos++) {
        g[pos] = s;
        s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)pos + 1u;
    }
    st.env[(int64_t)e * kEnvRec + ENV_MTPOS] = kMtN;
    st.env[(int64_t)e * kEnvRec + ENV_SPAWN] = SPAWN_NONE;
}

// rgb_from_grid (grid_util.py:164-175) of every env's current grid: a palette
// lookup per cell. Each thread writes 4 consecutive cells of the flat
// [N][H][W] image as three 4-byte stores (12 bytes at a 12-byte offset; cells
// past the last whole quad go byte by byte). HBM-bound: reads one
// ring byte and writes 3 bytes per cell, plus the 4-byte cur index per env.
struct RenderPal {
    uint8_t rgb[6 * kMaxSnakes * 3];
};

__device__ __forceinline__ uint32_t render_cell(const KCfg &c, const snake_state &st,
                                                const RenderPal &pal, long long x)
{
    const long long e = x / c.HW;
    const int cell = (int)(x - e * c.HW);
    const int cur = st.env[e * kEnvRec + ENV_CUR];
    const int v = st.grid[e * c.ring_bytes + (long long)cur * c.grid_stride + cell];
    const int code = v % 10, id = v / 10;
    if (code > 5 || id >= kMaxSnakes) return 0u;   // not a reachable grid value
    const uint8_t *p = pal.rgb + (code * kMaxSnakes + id) * 3;
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16);
}

__global__ void k_render(const KCfg c, const snake_state st, const RenderPal pal, uint8_t *rgb)
{
    const long long total = (long long)c.N * c.HW;
    const long long x0 = 4ll * ((long long)blockIdx.x * blockDim.x + threadIdx.x);
    if (x0 >= total) return;
    if (x0 + 4 <= total) {
        uint32_t q[4];
#pragma unroll
        for (int t = 0; t < 4; t++) q[t] = render_cell(c, st, pal, x0 + t);
        uint32_t *dst = reinterpret_cast<uint32_t *>(rgb + 3 * x0);
        dst[0] = q[0] | (q[1] << 24);
        dst[1] = (q[1] >> 8) | (q[2] << 16);
        dst[2] = (q[2] >> 16) | (q[3] << 8);
    } else {
        for (long long x = x0; x < x0 + 4 && x < total; x++) {
            const uint32_t q = render_cell(c, st, pal, x);
            rgb[3 * x] = (uint8_t)q;
            rgb[3 * x + 1] = (uint8_t)(q >> 8);
            rgb[3 * x + 2] = (uint8_t)(q >> 16);
        }
    }
}

// ------------------------------------------------------------- kernel timing
// Profiling aid (snake_timing_enable / snake_timing_read): pairs of timing events
// around each launch, resolved when read. Event objects are pooled.
namespace {
struct TimingRec {
    const char *name;
    hipEvent_t a, b;
};
std::mutex g_tmu;
bool g_timing = false;
int g_draw_wait_ticks = 200000;   // KCfg.draw_wait (snake_debug_set "draw_wait_ticks")
int g_spawn_delay_ticks = 0;      // KCfg.spawn_delay (snake_debug_set "spawn_delay_ticks")
int g_fuse_roles = 7;             // KCfg.fu_roles (snake_debug_set "fuse_roles", diagnostics)
#ifndef SNAKE_FUSED
#define SNAKE_FUSED 0
#endif
int g_fused = SNAKE_FUSED;        // the fused step where KCfg.fused allows it (snake_debug_set "fused")
std::vector<TimingRec> g_pending;
std::vector<hipEvent_t> g_pool;
std::map<std::string, std::pair<double, int64_t>> g_done;

hipEvent_t pooled_event()
{
    if (!g_pool.empty()) {
        hipEvent_t ev = g_pool.back();
        g_pool.pop_back();
        return ev;
    }
    hipEvent_t ev = nullptr;
    // timing only: no system-scope fence (cache write-back and invalidate) when
    // the event completes, which would delay the next kernel
    if (hipEventCreateWithFlags(&ev, hipEventDisableSystemFence) != hipSuccess) return nullptr;
    return ev;
}
}  // namespace

// Times the one launch (slaunch) made between its construction and close():
// the pair of pooled events rides on that launch (no-ops when timing is off).
struct TimedLaunch {
    const char *name;
    hipEvent_t a = nullptr, b = nullptr;
    TimedLaunch(const char *n, hipStream_t) : name(n)
    {
        std::lock_guard<std::mutex> g(g_tmu);
        if (!g_timing) return;
        a = pooled_event();
        b = a ? pooled_event() : nullptr;
        if (!b) {
            if (a) g_pool.push_back(a);
            a = nullptr;
            return;
        }
        t_ev0 = a;
        t_ev1 = b;
    }
    void close()
    {
        if (!a) return;
        t_ev0 = t_ev1 = nullptr;
        std::lock_guard<std::mutex> g(g_tmu);
        // (a failed launch records neither: check_launch reports it, the pair
        // goes back to the pool)
        if (hipPeekAtLastError() == hipSuccess) g_pending.push_back({name, a, b});
        else {
            g_pool.push_back(a);
            g_pool.push_back(b);
        }
        a = nullptr;
    }
    ~TimedLaunch() { close(); }
};

// Every launch runs with the caller stream's device current: the side stream and
// events are created on it, and a SnakeVecEnv on cuda:1 works whatever device the
// calling thread has current (restored on return).
struct DeviceGuard {
    int dev = -1, prev = -1;
    explicit DeviceGuard(hipStream_t s)
    {
        if (hipGetDevice(&prev) != hipSuccess) { set_error("hipGetDevice failed"); return; }
        if (s == nullptr) { dev = prev; return; }
        if (hipStreamGetDevice(s, &dev) != hipSuccess) {
            set_error("hipStreamGetDevice failed");
            dev = -1;
            return;
        }
        if (dev != prev && hipSetDevice(dev) != hipSuccess) {
            set_error("hipSetDevice(%d) failed", dev);
            dev = -1;
        }
    }
    ~DeviceGuard()
    {
        if (prev >= 0 && dev >= 0 && dev != prev) (void)hipSetDevice(prev);
    }
};

// ---------------------------------------------------------------- launchers
static int check_launch(const char *what)
{
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        set_error("%s launch failed: %s", what, hipGetErrorString(err));
        return SNAKE_E_LAUNCH;
    }
    return SNAKE_OK;
}

// The background stream's events only order kernels of one device: no
// system-scope fence (that would write the L2s back for a host that never looks).
constexpr unsigned kJoinFlags = hipEventDisableTiming | hipEventDisableSystemFence;

// Background spawn-ahead (KCfg.bg) per state (keyed by its env records): the
// stream k_spawn runs on, the event the caller's stream records after k_logic
// (k_spawn's start), the event recorded after the last k_spawn of each queue
// set, the step counter whose parity picks the queue set. Created by the
// state's first step, destroyed by snake_release.
// One background stream per queue set (round 5): a set's k_spawn only waits for
// that set's previous one, so consecutive steps' spawn kernels may overlap --
// with one stream they queued behind each other (a 40x40 job takes about a
// step) and k_logic found its set's previous kernel unfinished in ~21 % of
// cfg5's steps, queued nothing, and the next step's resets drew inline.
constexpr int kBgStreams = 2;
struct BgCtx {
    // (two streams for the four queue sets, set p on stream p % 2: every
    // stream takes one of the process's hardware queues -- GPU_MAX_HW_QUEUES,
    // 4 by default -- and with four background streams the caller's stream
    // shared one with a spawn kernel: cfg5 0.0811 -> 0.0980 ms, round 6)
    hipStream_t x[kBgStreams] = {};
    hipEvent_t fork = nullptr;
    hipEvent_t done[kQSets] = {};
    uint64_t steps = 0;
    bool pending[kQSets] = {};
    uint32_t launched[kQSets] = {};   // k_spawn launches per queue set (KCfg.spawn_gate)
};
static std::mutex g_bgmu;
static std::map<const void *, BgCtx> g_bg;
// The fused step's per-state epoch (k_step): the number of k_step launches of
// the state so far; its flag area is zeroed on the state's first fused step.
static std::map<const void *, uint32_t> g_fu;

static void destroy_bg(BgCtx &c)
{
    for (hipStream_t x : c.x)
        if (x) (void)hipStreamSynchronize(x);   // (its last k_spawn)
    if (c.fork) (void)hipEventDestroy(c.fork);
    for (hipEvent_t ev : c.done)
        if (ev) (void)hipEventDestroy(ev);
    for (hipStream_t x : c.x)
        if (x) (void)hipStreamDestroy(x);
    c = BgCtx();
}

static BgCtx *bg_ctx(const snake_state &st, bool create)
{
    std::lock_guard<std::mutex> g(g_bgmu);
    auto it = g_bg.find(st.env);
    if (it != g_bg.end()) return &it->second;
    if (!create) return nullptr;
    BgCtx c;
    bool ok = true;
    for (int p = 0; p < kBgStreams && ok; p++)
        ok = hipStreamCreateWithFlags(&c.x[p], hipStreamNonBlocking) == hipSuccess;
    for (int p = 0; p < kQSets && ok; p++)
        ok = hipEventCreateWithFlags(&c.done[p], kJoinFlags) == hipSuccess;
    // (the fork event rides on k_logic's dispatch as its stop event, like the
    // timing events: a timing-capable event without the system fence)
    if (!ok || hipEventCreateWithFlags(&c.fork, hipEventDisableSystemFence) != hipSuccess) {
        destroy_bg(c);
        set_error("background stream / event creation failed");
        return nullptr;
    }
    return &g_bg.emplace(st.env, c).first->second;   // (std::map: the address stays valid)
}

// `stream` waits for the state's last background spawn kernel (if any).
int wait_background(const snake_state &st, void *stream)
{
    BgCtx *b = bg_ctx(st, false);
    if (!b) return SNAKE_OK;
    for (int p = 0; p < kQSets; p++)
        if (b->pending[p] && hipStreamWaitEvent((hipStream_t)stream, b->done[p], 0) != hipSuccess) {
            set_error("waiting for the background spawn kernel failed");
            return SNAKE_E_LAUNCH;
        }
    return SNAKE_OK;
}

// The state's background context (snake_release): its last spawn kernel
// waited for on the host, its stream and events destroyed, the entry erased,
// so an allocation that later reuses the same env address starts afresh.
int release_background(const snake_state &st)
{
    BgCtx c;
    {
        std::lock_guard<std::mutex> g(g_bgmu);
        g_fu.erase(st.env);
        auto it = g_bg.find(st.env);
        if (it == g_bg.end()) return SNAKE_OK;
        c = it->second;
        g_bg.erase(it);
    }
    DeviceGuard dg(c.x[0]);   // (the streams' device current while they are destroyed)
    destroy_bg(c);
    return dg.dev < 0 ? SNAKE_E_LAUNCH : SNAKE_OK;
}

int launch_seed(const KCfg &k, const snake_state &st, uint32_t base_seed, int64_t env_offset,
                void *stream)
{
    const int threads = 256, blocks = (k.N + threads - 1) / threads;
    DeviceGuard dg((hipStream_t)stream);
    if (dg.dev < 0) return SNAKE_E_LAUNCH;
    if (int rc = wait_background(st, stream)) return rc;
    slaunch(k_seed, dim3(blocks), dim3(threads), 0, (hipStream_t)stream, k, st,
                       base_seed, (long long)env_offset);
    return check_launch("k_seed");
}

int launch_render(const KCfg &k, const snake_state &st, const uint8_t *palette, uint8_t *rgb,
                  void *stream)
{
    RenderPal pal;
    memcpy(pal.rgb, palette, sizeof(pal.rgb));
    DeviceGuard dg((hipStream_t)stream);
    if (dg.dev < 0) return SNAKE_E_LAUNCH;
    const long long quads = ((long long)k.N * k.HW + 3) / 4;
    const int threads = 256;
    const long long blocks = (quads + threads - 1) / threads;
    slaunch(k_render, dim3((unsigned)blocks), dim3(threads), 0, (hipStream_t)stream, k, st,
                       pal, rgb);
    return check_launch("k_render");
}

int launch_reset(const KCfg &k, const snake_state &st, const uint8_t *mask, const snake_out &o,
                 void *stream)
{
    const dim3 grid(k.link_in_lds ? k.N : k.reset_slots), block(kWave);
    DeviceGuard dg((hipStream_t)stream);
    if (dg.dev < 0) return SNAKE_E_LAUNCH;
    if (int rc = wait_background(st, stream)) return rc;
    TimedLaunch tl("k_reset", (hipStream_t)stream);
    const KArgs a{k, st, o, mask};
    const hipStream_t s = (hipStream_t)stream;
    if (k.link32) {
        if (k.S <= 4) slaunch((k_reset<4, 2>), grid, block, k.lds_bytes, s, a);
        else if (k.S <= 8) slaunch((k_reset<8, 2>), grid, block, k.lds_bytes, s, a);
        else slaunch((k_reset<16, 2>), grid, block, k.lds_bytes, s, a);
    } else if (k.link_in_lds) {
        if (k.S <= 4) slaunch((k_reset<4, 1>), grid, block, k.lds_bytes, s, a);
        else if (k.S <= 8) slaunch((k_reset<8, 1>), grid, block, k.lds_bytes, s, a);
        else slaunch((k_reset<16, 1>), grid, block, k.lds_bytes, s, a);
    } else {
        if (k.S <= 4) slaunch((k_reset<4, 0>), grid, block, k.lds_bytes, s, a);
        else if (k.S <= 8) slaunch((k_reset<8, 0>), grid, block, k.lds_bytes, s, a);
        else slaunch((k_reset<16, 0>), grid, block, k.lds_bytes, s, a);
    }
    tl.close();
    return check_launch("k_reset");
}

// k_post<MS(S), NPF, RO, JL> (see k_post)
template <int MS, bool RO, int JL>
static void launch_post(const KCfg &k, const KArgs &a, int npf, dim3 grid, int lds, hipStream_t s)
{
    const dim3 block(kWave);
    if (npf == 0) slaunch((k_post<MS, 0, RO, JL>), grid, block, lds, s, a);
    else if (npf == -2) slaunch((k_post<MS, -2, RO, JL>), grid, block, lds, s, a);
    else if (npf == -8) slaunch((k_post<MS, -8, RO, JL>), grid, block, lds, s, a);
    else if (npf == 1) slaunch((k_post<MS, 1, RO, JL>), grid, block, lds, s, a);
    else if (npf == 2) slaunch((k_post<MS, 2, RO, JL>), grid, block, lds, s, a);
    else slaunch((k_post<MS, 8, RO, JL>), grid, block, lds, s, a);
}

template <bool RO, int JL>
static void launch_post_s(const KCfg &k, const KArgs &a, int npf, dim3 grid, int lds, hipStream_t s)
{
    if (k.S <= 4) launch_post<4, RO, JL>(k, a, npf, grid, lds, s);
    else if (k.S <= 8) launch_post<8, RO, JL>(k, a, npf, grid, lds, s);
    else launch_post<16, RO, JL>(k, a, npf, grid, lds, s);
}

// k_autoreset<MS(S), RO, JL(k.link_in_lds)> (every-step mode: resets only)
static void launch_autoreset_ro(const KCfg &k, const KArgs &a, dim3 grid, hipStream_t s)
{
    const dim3 block(kWave);
    if (k.link_in_lds) {
        if (k.S <= 4) slaunch((k_autoreset<4, true, 1>), grid, block, k.lds_bytes, s, a);
        else if (k.S <= 8) slaunch((k_autoreset<8, true, 1>), grid, block, k.lds_bytes, s, a);
        else slaunch((k_autoreset<16, true, 1>), grid, block, k.lds_bytes, s, a);
    } else {
        if (k.S <= 4) slaunch((k_autoreset<4, true, 0>), grid, block, k.lds_bytes, s, a);
        else if (k.S <= 8) slaunch((k_autoreset<8, true, 0>), grid, block, k.lds_bytes, s, a);
        else slaunch((k_autoreset<16, true, 0>), grid, block, k.lds_bytes, s, a);
    }
}

// snake_step: k_logic, then (all-done auto-reset) the shared phase as ONE launch
// on the caller's stream -- k_post, or k_post_lean on boards with four-wave lean
// encodes -- with, on background spawn-ahead boards, k_spawn forked onto the
// state's background stream after k_logic and not joined.
int launch_step(const KCfg &k0, const snake_state &st, const int8_t *actions, const snake_out &o,
                void *stream)
{
    KCfg k = k0;
    k.diag = g_timing ? 1 : 0;
    k.draw_wait = g_draw_wait_ticks;
    k.spawn_delay = g_spawn_delay_ticks;
    k.fu_roles = g_fuse_roles;
    const hipStream_t sm = (hipStream_t)stream;
    DeviceGuard dg(sm);
    if (dg.dev < 0) return SNAKE_E_LAUNCH;
    const int ms = k.logic_ms, epw = kWave / ms;   // envs per k_logic wave
    const int lds_logic = k.lds_logic;
    const dim3 g1(k.N), gl((k.N + epw - 1) / epw), gr(k.reset_slots), block(kWave);
    // everything that can fail before k_logic fills this step's queue set
    BgCtx *bgc = nullptr;
    if (k.bg) {   // background spawn-ahead: this step's queue set; k_logic queues
                  // spawn-ahead jobs into it only if the spawn kernels launched on
                  // it so far have finished (kQSpGen), the stream never waits
                  // (the wait cost cfg5 0.1026 -> 0.1136 ms per step)
        if (!(bgc = bg_ctx(st, true))) return SNAKE_E_LAUNCH;
        k.qpar = (int)(bgc->steps % kQSets);
        k.spawn_gate = bgc->launched[k.qpar];
    }
    if (k.fused && g_fused) {   // the whole step as one launch (k_step)
        uint32_t ep;
        bool fresh = false;
        {
            std::lock_guard<std::mutex> g(g_bgmu);
            auto it = g_fu.find(st.env);
            if (it == g_fu.end()) { it = g_fu.emplace(st.env, 0u).first; fresh = true; }
            ep = it->second;
        }
        if (fresh && hipMemsetAsync(st.resetq + k.fu_ldone, 0, sizeof(int) * fused_words(k.N), sm) != hipSuccess) {
            set_error("zeroing the fused step's flags failed");
            return SNAKE_E_LAUNCH;
        }
        k.epoch = ep + 1;
        const int npw = (k.fs * k.HW / 4 + kWave - 1) / kWave;
        const dim3 gf(k.nlg + k.reset_slots + (k.N + 3) / 4), bf(kWave);
        const int lds_f = std::max(k.lds_logic, std::max(k.lds_bytes, k.lds_tbl_bytes));
        const KArgs fa{k, st, o, actions};
        TimedLaunch tf("k_step", sm);
        auto go = [&](auto msc, auto npwc) {
            constexpr int MS = decltype(msc)::value, NPW = decltype(npwc)::value;
            if (k.link32) slaunch((k_step<MS, NPW, 2>), gf, bf, lds_f, sm, fa);
            else slaunch((k_step<MS, NPW, 1>), gf, bf, lds_f, sm, fa);
        };
        using I2 = std::integral_constant<int, 2>;
        using I4 = std::integral_constant<int, 4>;
        using I8 = std::integral_constant<int, 8>;
        if (ms == 4) { if (npw <= 2) go(I4{}, I2{}); else go(I4{}, I8{}); }
        else { if (npw <= 2) go(I8{}, I2{}); else go(I8{}, I8{}); }
        tf.close();
        if (int rc2 = check_launch("k_step")) return rc2;
        std::lock_guard<std::mutex> g(g_bgmu);
        g_fu[st.env] = ep + 1;
        return SNAKE_OK;
    }
    TimedLaunch t1("k_logic", sm);
    // Background spawn-ahead: the fork onto the background stream is k_logic's
    // own dispatch -- its stop event (the timing event when the launch is timed)
    // -- not an event record of its own on the caller's stream: that marker
    // packet stood between k_logic and k_post, 5.3 us of idle GPU per step at
    // 8 192 envs (round 6 kernel trace).
    hipEvent_t fork_ev = nullptr;
    if (bgc) {
        if (!t_ev1) t_ev1 = bgc->fork;
        fork_ev = t_ev1;
    }
    const KArgs la{k, st, o, actions};
    // four waves (groups) per workgroup where their LDS fits (KCfg.logic_wpb):
    // k_logic cfg4 20.4 -> 19.4 us, cfg5 21.9 -> 21.1 against one (round 4)
    auto launch_logic = [&](auto wpb) {
        constexpr int WPB = decltype(wpb)::value;
        const dim3 glb((gl.x + WPB - 1) / WPB), blb(kWave * WPB);
        if (k.bg) {
            if (ms == 4) slaunch((k_logic<4, WPB, true>), glb, blb, WPB * lds_logic, sm, la);
            else if (ms == 8) slaunch((k_logic<8, WPB, true>), glb, blb, WPB * lds_logic, sm, la);
            else slaunch((k_logic<16, WPB, true>), glb, blb, WPB * lds_logic, sm, la);
        } else {
            if (ms == 4) slaunch((k_logic<4, WPB, false>), glb, blb, WPB * lds_logic, sm, la);
            else if (ms == 8) slaunch((k_logic<8, WPB, false>), glb, blb, WPB * lds_logic, sm, la);
            else slaunch((k_logic<16, WPB, false>), glb, blb, WPB * lds_logic, sm, la);
        }
    };
    if (k.logic_wpb == 4) launch_logic(std::integral_constant<int, 4>{});
    else launch_logic(std::integral_constant<int, 1>{});
    if (bgc && fork_ev == bgc->fork) t_ev1 = nullptr;
    t1.close();
    int rc = check_launch("k_logic");
    if (rc) return rc;
    // From here on k_logic has filled this step's queue set: a failure zeroes
    // its counters, so the next step does not run this step's queues. Once
    // k_spawn is launched it owns the set's spawn counters (it reads them and
    // re-zeroes them at its end): only the reset counters are zeroed
    // then -- queue 0's shard counts and the claim / done counters.
    bool spawn_launched = false;
    auto fail = [&](int r) {
        int *qc = st.resetq + (int64_t)k.qpar * (kNumQ * kQShards * k.q_cap + kQCounters) +
                  kNumQ * kQShards * k.q_cap;
        if (!spawn_launched) {
            // (ordered after the set's previous k_spawn, which may still use its
            // spawn and claim counters on its background stream)
            if (bgc && bgc->pending[k.qpar]) (void)hipStreamWaitEvent(sm, bgc->done[k.qpar], 0);
            (void)hipMemsetAsync(qc, 0, sizeof(int) * kQSpGen * kQSpread, sm);   // (not the finished count)
        } else {
            (void)hipMemsetAsync(qc, 0, sizeof(int) * kQShards * kQSpread, sm);
            (void)hipMemsetAsync(qc + kQClaim * kQSpread, 0, sizeof(int) * (kQDone + 1 - kQClaim) * kQSpread, sm);
        }
        return r;
    };
    const KArgs a{k, st, o, nullptr};
    if (k.autoreset == 2) {   // every env resets (the resets write the obs), then the
                              // encodes of the envs rejected for an invalid action
        TimedLaunch t2("k_autoreset", sm);
        launch_autoreset_ro(k, a, gr, sm);
        t2.close();
        if ((rc = check_launch("k_autoreset"))) return fail(rc);
        TimedLaunch t3("k_encode", sm);
        slaunch(k_encode, g1, block, k.lds_obs_bytes, sm, k, st, o);
        t3.close();
        return check_launch("k_encode");
    }
    if (!k.autoreset) {
        TimedLaunch t3("k_encode", sm);
        slaunch(k_encode, g1, block, k.lds_obs_bytes, sm, k, st, o);
        t3.close();
        return check_launch("k_encode");
    }
    if (bgc) {
        // this step's spawn kernel on the background stream once k_logic has
        // passed (its dispatch's stop event, above); not joined (k_logic two
        // steps later only queues into the set once it has finished)
        hipStream_t bx = bgc->x[k.qpar % kBgStreams];
        if (hipStreamWaitEvent(bx, fork_ev, 0) != hipSuccess) {
            set_error("fork to the background stream failed");
            return fail(SNAKE_E_LAUNCH);
        }
        KCfg ks = k;
        ks.lds_link = 0;   // (only the draw record)
        const int lds_sp = (int)(((int64_t)2 * (k.n_cand + kWave) + 15) / 16 * 16);
        const dim3 gs(k.spawn_slots);
        TimedLaunch t4("k_spawn", bx);
        const KArgs sa{ks, st, o, nullptr};
        if (k.S <= 4) slaunch(k_spawn<4>, gs, block, lds_sp, bx, sa);
        else if (k.S <= 8) slaunch(k_spawn<8>, gs, block, lds_sp, bx, sa);
        else slaunch(k_spawn<16>, gs, block, lds_sp, bx, sa);
        t4.close();
        if ((rc = check_launch("k_spawn"))) return fail(rc);
        // (counted as soon as it is launched: its last worker adds one to the
        // set's finished count whatever fails after this point)
        spawn_launched = true;
        bgc->launched[k.qpar]++;
        bgc->steps++;
        if (hipEventRecord(bgc->done[k.qpar], bx) != hipSuccess) {
            // (pending / done[] would not cover this k_spawn, which writes
            // records, env word 4 and the set's counters: wait for it here so
            // that snake_sync and the next steps need not)
            (void)hipStreamSynchronize(bx);
            set_error("background spawn event failed");
            return fail(SNAKE_E_LAUNCH);
        }
        bgc->pending[k.qpar] = true;
    }
    TimedLaunch t2("k_post", sm);
    if (k.lean) {
        // four workers per workgroup, then the four-wave lean encodes
        const dim3 gp((k.reset_slots + 3) / 4 + (k.N + k.enc_per_wave - 1) / k.enc_per_wave);
        const int lds_p = std::max(4 * k.lds_worker, k.tbl ? k.lds_tbl_bytes : k.lds_lean_bytes);
        if (k.tbl) {   // (the table encode in four-wave workgroups)
            if (k.bg) {
                if (k.S <= 4) slaunch((k_post_lean<4, true, true>), gp, dim3(256), lds_p, sm, a);
                else if (k.S <= 8) slaunch((k_post_lean<8, true, true>), gp, dim3(256), lds_p, sm, a);
                else slaunch((k_post_lean<16, true, true>), gp, dim3(256), lds_p, sm, a);
            } else {
                if (k.S <= 4) slaunch((k_post_lean<4, false, true>), gp, dim3(256), lds_p, sm, a);
                else if (k.S <= 8) slaunch((k_post_lean<8, false, true>), gp, dim3(256), lds_p, sm, a);
                else slaunch((k_post_lean<16, false, true>), gp, dim3(256), lds_p, sm, a);
            }
        } else if (k.bg) {
            if (k.S <= 4) slaunch((k_post_lean<4, true, false>), gp, dim3(256), lds_p, sm, a);
            else if (k.S <= 8) slaunch((k_post_lean<8, true, false>), gp, dim3(256), lds_p, sm, a);
            else slaunch((k_post_lean<16, true, false>), gp, dim3(256), lds_p, sm, a);
        } else {
            if (k.S <= 4) slaunch((k_post_lean<4, false, false>), gp, dim3(256), lds_p, sm, a);
            else if (k.S <= 8) slaunch((k_post_lean<8, false, false>), gp, dim3(256), lds_p, sm, a);
            else slaunch((k_post_lean<16, false, false>), gp, dim3(256), lds_p, sm, a);
        }
    } else {
        // the workers, then the encodes: NPF = 16-byte ring chunks per lane the
        // two-env encode keeps in flight, 0 = one env per block
        const int epw2 = k.enc_per_wave, n16 = k.ring_bytes >> 4;
        const int npw = (k.fs * k.HW / 4 + kWave - 1) / kWave;   // frame dwords per lane (table encode)
        const int npf = k.tbl ? (npw <= 2 ? -2 : -8)
                              : (epw2 <= 1 ? 0 : (n16 <= kWave ? 1 : (n16 <= 2 * kWave ? 2 : 8)));
        const int enc_blocks = npf == 0 ? k.N : (k.N + epw2 - 1) / epw2;
        const dim3 gp(k.reset_slots + enc_blocks);
        const int lds_p = std::max(k.lds_bytes, k.tbl ? k.lds_tbl_bytes : k.lds_obs_bytes);
        if (k.bg) launch_post_s<true, 1>(k, a, npf, gp, lds_p, sm);   // (background boards keep the LDS record)
        else if (k.link32) launch_post_s<false, 2>(k, a, npf, gp, lds_p, sm);
        else if (k.link_in_lds) launch_post_s<false, 1>(k, a, npf, gp, lds_p, sm);
        else launch_post_s<false, 0>(k, a, npf, gp, lds_p, sm);
    }
    t2.close();
    if ((rc = check_launch("k_post"))) return fail(rc);
#ifdef SNAKE_DIAG_ENC2
    // Diagnostic timing build: k_post once more with idle workers (aux set), so
    // the encodes alone are timed ("k_encode") with the same launch shape, LDS
    // and registers; they rewrite the same observations.
    if (!k.lean) {
        const int epw2 = k.enc_per_wave, n16 = k.ring_bytes >> 4;
        const int npw = (k.fs * k.HW / 4 + kWave - 1) / kWave;
        const int npf = k.tbl ? (npw <= 2 ? -2 : -8)
                              : (epw2 <= 1 ? 0 : (n16 <= kWave ? 1 : (n16 <= 2 * kWave ? 2 : 8)));
        const int enc_blocks = npf == 0 ? k.N : (k.N + epw2 - 1) / epw2;
        const dim3 gp(k.reset_slots + enc_blocks);
        const int lds_p = std::max(k.lds_bytes, k.tbl ? k.lds_tbl_bytes : k.lds_obs_bytes);
        const KArgs a2{k, st, o, (const void *)1};
        TimedLaunch t5("k_encode", sm);
        if (k.link32) launch_post_s<false, 2>(k, a2, npf, gp, lds_p, sm);
        else launch_post_s<false, 1>(k, a2, npf, gp, lds_p, sm);
        t5.close();
    }
#endif
    return SNAKE_OK;
}

}  // namespace snake

extern "C" int snake_timing_enable(int on)
{
    std::lock_guard<std::mutex> g(snake::g_tmu);
    snake::g_timing = on != 0;
    return SNAKE_OK;
}

#ifdef SNAKE_FUSE_DEBUG
extern "C" int snake_debug_fdbg(unsigned long long *out)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(snake::g_fdbg), sizeof(unsigned long long) * 64) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int snake_debug_set(const char *name, long long value)
{
    if (name && value >= 0 && value <= INT_MAX) {
        std::lock_guard<std::mutex> g(snake::g_tmu);
        if (!strcmp(name, "draw_wait_ticks")) { snake::g_draw_wait_ticks = (int)value; return SNAKE_OK; }
        if (!strcmp(name, "spawn_delay_ticks")) { snake::g_spawn_delay_ticks = (int)value; return SNAKE_OK; }
        if (!strcmp(name, "fuse_roles")) { snake::g_fuse_roles = (int)value; return SNAKE_OK; }
        if (!strcmp(name, "fused")) { snake::g_fused = value ? 1 : 0; return SNAKE_OK; }
    }
    snake::set_error("snake_debug_set: unknown knob or value out of range");
    return SNAKE_E_ARG;
}

extern "C" int snake_timing_read(const char *kernel, double *total_ms, int64_t *count)
{
    if (!kernel || !total_ms || !count) {
        snake::set_error("snake_timing_read: NULL argument");
        return SNAKE_E_ARG;
    }
    const bool one = !strcmp(kernel, "resets") || !strcmp(kernel, "resets_timed");
    const void *sym = !strcmp(kernel, "resets") ? (const void *)&snake::g_resets_run
                    : !strcmp(kernel, "resets_timed") ? (const void *)&snake::g_resets_timed
                    : !strcmp(kernel, "spawn_hits") ? (const void *)snake::g_spawn_hits
                    : !strcmp(kernel, "spawn_jobs") ? (const void *)snake::g_spawn_jobs
                    : !strcmp(kernel, "spawn_void") ? (const void *)snake::g_spawn_void
                    : !strcmp(kernel, "reset_partial") ? (const void *)snake::g_reset_part
                    : !strcmp(kernel, "respawn_slow") ? (const void *)snake::g_resp_slow
                    : !strcmp(kernel, "respawn_slow2") ? (const void *)snake::g_resp_slow2
                    : !strcmp(kernel, "gate_shut") ? (const void *)snake::g_gate_shut
                    : !strcmp(kernel, "draw_wait") ? (const void *)snake::g_draw_wait
                    : !strcmp(kernel, "draw_timeout") ? (const void *)snake::g_draw_timeout
                    : !strcmp(kernel, "fused_timeout") ? (const void *)snake::g_fused_timeout : nullptr;
    if (sym) {
        const int n = one ? 1 : snake::kDiagSlots * snake::kDiagSpread;
        std::vector<unsigned long long> v(n, 0ull), z(n, 0ull);
        if (hipMemcpyFromSymbol(v.data(), sym, n * sizeof(unsigned long long)) != hipSuccess ||
            hipMemcpyToSymbol(sym, z.data(), n * sizeof(unsigned long long)) != hipSuccess) {
            snake::set_error("snake_timing_read: reading the reset counter failed");
            return SNAKE_E_LAUNCH;
        }
        unsigned long long t = 0;
        for (unsigned long long x : v) t += x;
        *total_ms = 0.0;
        *count = (int64_t)t;
        return SNAKE_OK;
    }
    std::lock_guard<std::mutex> g(snake::g_tmu);
    for (const auto &r : snake::g_pending) {
        float ms = 0.f;
        if (hipEventSynchronize(r.b) != hipSuccess || hipEventElapsedTime(&ms, r.a, r.b) != hipSuccess) {
            snake::set_error("snake_timing_read: event query failed");
            return SNAKE_E_LAUNCH;
        }
        auto &d = snake::g_done[r.name];
        d.first += ms;
        d.second += 1;
        snake::g_pool.push_back(r.a);
        snake::g_pool.push_back(r.b);
    }
    snake::g_pending.clear();
    auto it = snake::g_done.find(kernel);
    *total_ms = it == snake::g_done.end() ? 0.0 : it->second.first;
    *count = it == snake::g_done.end() ? 0 : it->second.second;
    if (it != snake::g_done.end()) snake::g_done.erase(it);
    return SNAKE_OK;
}

#ifdef SNAKE_DRAWBENCH
// (diagnostic build only: the isolated draw / attempt benchmarks and the
// cooperative four-wave draws they compare against, scripts/microbench/)
#include "../../scripts/microbench/drawbench.inc"
#endif

#ifdef SNAKE_STAMPS
// out: 16 * 8192 per-wave phase realtimes of the last k_logic (g_wphase)
extern "C" int snake_debug_wphase(unsigned long long *out)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(snake::g_wphase), sizeof(unsigned long long) * 16 * snake::kWaveTimes) ==
                   hipSuccess ? 0 : -1;
}

// out: the reset workers' items of the launches since the last call (4 words
// each, see g_items), at most cap; returns their number
extern "C" int snake_debug_items(unsigned long long *out, int cap)
{
    unsigned n = 0, z = 0;
    if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(snake::g_nitems), sizeof n) != hipSuccess) return -1;
    n = std::min<unsigned>(n, (unsigned)std::min(cap, snake::kItems));
    if (n && hipMemcpyFromSymbol(out, HIP_SYMBOL(snake::g_items), sizeof(unsigned long long) * 4 * n) != hipSuccess)
        return -1;
    if (hipMemcpyToSymbol(HIP_SYMBOL(snake::g_nitems), &z, sizeof z) != hipSuccess) return -1;
    return (int)n;
}

// out: 64 phase stamps of block 0, 2 * 8192 k_logic wave start/end realtimes,
// 2 * 40960 k_post block start/end realtimes
extern "C" int snake_debug_stamps(unsigned long long *out)
{
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(snake::g_stamps), sizeof(unsigned long long) * 64) != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out + 64, HIP_SYMBOL(snake::g_wavetime),
                            sizeof(unsigned long long) * 2 * snake::kWaveTimes) != hipSuccess) return -1;
    return hipMemcpyFromSymbol(out + 64 + 2 * snake::kWaveTimes, HIP_SYMBOL(snake::g_posttime),
                               sizeof(unsigned long long) * 2 * snake::kPostTimes) == hipSuccess ? 0 : -1;
}
#endif
