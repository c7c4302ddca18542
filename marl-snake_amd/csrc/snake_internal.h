// snake_internal.h -- launch-side configuration shared by snake_capi.cpp and
// snake_kernels.hip (not part of the C-ABI).
#pragma once
#include <stdint.h>

#include "../../include/snake_env.h"

namespace snake {

constexpr int kWave = 64;
constexpr int kMtN = 624;
constexpr int kMaxSnakes = 16;
constexpr int kMaxFruits = 64;
constexpr int kEnvRec = 8;          // int32 words per env record
constexpr int kJarrLdsMax = 36864;  // bytes of a reset's u16 draw record kept in LDS
constexpr int kLdsLimit = 160 * 1024;   // LDS per workgroup (gfx950)
// concurrent reset workers (global link tables): 8 per CU; with k_post 2 048 beat
// 2 560 (round 2: cfg3 0.0905 -> 0.0892 ms; 1 536 0.106); round 4: 2 560 and 3 072
// equal (every spawn-ahead job a first job: cfg3 0.0838 / 0.0837), 1 792 0.1016
constexpr int kResetSlots = 2048;
constexpr int kQShards = 64;        // auto-reset queue shards (k_logic block % 64)
constexpr int kStageMax = 8192;     // bytes of staged observation per encode group
constexpr int kSpawnStride = 672;   // u32 words per spawn-ahead record: key, pos, the poses' cells
constexpr int kSpawnPos = 624;      // record word: MT position after the recorded attempts
constexpr int kSpawnCells = 625;    // record words [625, 657): the S*L spawn cells, u16, two per word
// Queue counters (zero between steps). Every counter sits in a line of its own
// (kQSpread words apart): same-line device-scope atomics from thousands of
// waves serialise at the memory side.
constexpr int kQSpread = 32;
constexpr int kClaimShards = 16;    // claim counters: worker w claims on shard w % 16
constexpr int kNumQ = 3;            // queues: 0 resets, 1 urgent spawn-ahead (<= 1 live snake), 2 other spawn-ahead
constexpr int kQClaim = kNumQ * kQShards;             // counter index of claim shard 0
constexpr int kQDone = kQClaim + kClaimShards;        // counter index: claim shards drained
constexpr int kQSpClaim = kQDone + 1;                 // background spawn kernel (k_spawn): claim shard 0
constexpr int kQSpDone = kQSpClaim + kClaimShards;    // k_spawn: claim shards drained
// k_spawn launches on this set that have finished (each one's last worker adds
// one after re-zeroing the set's spawn counters; never zeroed): k_logic queues
// spawn-ahead jobs into the set only when it equals KCfg.spawn_gate, the count
// launched so far, instead of the step waiting for the background stream
constexpr int kQSpGen = kQSpDone + 1;
constexpr int kQCount = kQSpGen + 1;                  // counters
constexpr int kQCounters = kQCount * kQSpread;        // words
// The queues and counters exist kQSets times (the step count mod kQSets,
// KCfg.qpar): with the background spawn kernel a step's spawn-ahead queues are
// still being read while the next steps' k_logic fill the other sets; a set is
// refilled only once its previous spawn kernel has finished (kQSpGen). Four
// sets (round 6; two until then): a spawn kernel may run for three steps before
// it holds up the queueing, so its jobs can afford more than one attempt.
#ifndef SNAKE_QSETS
#define SNAKE_QSETS 4
#endif
constexpr int kQSets = SNAKE_QSETS;   // (2 or 4: the status word's two buffer bits)
static_assert(kQSets == 2 || kQSets == 4, "two or four queue sets");
constexpr int kQGenBits = 6;        // spawn queue entry (background mode): env | generation << 26

// env record words (6, 7 unused)
enum { ENV_ALIVE = 0, ENV_EPLEN = 1, ENV_CUR = 2, ENV_MTPOS = 3, ENV_SPAWN = 4, ENV_FAIL = 5 };
// spawn-ahead status word (env word ENV_SPAWN): bits 0-1 the status, bits 2-3 the
// record buffer holding the record (background spawn-ahead keeps one per queue
// set and env), bits 4-31 the record's generation (bumped by every MT draw that
// voids it)
constexpr int kSpawnBufShift = 2, kSpawnGenShift = 4;
// DRAWING (background spawn-ahead only): a k_spawn job is drawing the record
// (from the env's own MT state or the partial record the buffer bit points at)
enum { SPAWN_NONE = 0, SPAWN_PARTIAL = 1, SPAWN_READY = 2, SPAWN_DRAWING = 3 };

// Everything a kernel needs, by value (a kernel argument).
struct KCfg {
    int N;
    int H, W, HW, S, L, vr, fs, observer, num_fruits, coop, autoreset;
    int oh, ow, units;          // units = S*oh*ow*fs (one unit = 8 obs bytes)
    int grid_stride, ring_cap, n_cand;
    int cs;                     // cells per lane when a wave sweeps the grid
    int ring_bytes;             // fs * grid_stride (the grid ring of one env)
    // step of 128 units expressed in the mixed radix (fs, ow, oh, S)
    int adv_f, adv_j, adv_i, adv_k;
    // dynamic LDS carve (bytes, 16-aligned)
    int lds_frames, lds_centers, lds_fruit, lds_link, lds_bytes, link_in_lds;
    // link_in_lds: the draws record j_i (u16 per i) in LDS at lds_link; else each
    // worker's u32 link table in global scratch, link_stride = round4(n_cand) + 64
    // per-lane dummies entries per table
    int link_stride;
    int link32;                 // the LDS link table as u32 (ds_min) + pointer chase instead of the u16 record + scan (JL = 2)
    int lds_obs_bytes;          // LDS of k_encode: no reset worker state
    // row-wise encode through an LDS staging buffer (encode_rows): snakes per
    // staged group (0: direct encode), the buffer, and magic reciprocals of
    // fs*oh and oh (x / d == umulhi(x, m) for the row indices used)
    int enc_group, lds_stage;
    uint32_t mag_fsoh, mag_oh;
    uint32_t mag_W;             // x / W == umulhi(x, mag_W) for cell indices x < H*W
    uint32_t mag_n16;           // q / (grid_stride/16) == umulhi(q, mag_n16) for q < 2^32/n16
    int reset_slots;            // min(N, kResetSlots)
    int logic_ms;               // k_logic's lanes per env (its MS: 4, 8 or 16, >= S)
    int lds_logic;              // k_logic's LDS bytes per wave: the group's frames, the fruit buffer, respawn scratch
    int logic_wpb;              // k_logic's waves per workgroup (4, or 1 where 4 * lds_logic exceeds kLdsLimit)
    int q_envs_per_block;       // envs per k_logic block (64 / logic_ms)
    int q_cap;                  // queue entries per shard
    int spawn_thr;              // queue spawn-ahead when <= this many snakes live (-1: off)
    int spawn_prio;             // wave priority of the spawn-ahead jobs (resets: 3)
    int encode_prio;            // wave priority of k_encode (beside the reset workers)
    int diag;                   // count spawn-ahead hits/jobs and resets (while timing is enabled)
    int enc_per_wave;           // envs per encode wave of k_post (1: encode_one, else encode_multi with prefetch)
    int bg;                     // 1: spawn-ahead jobs in the background kernel k_spawn (not in the step)
    int lds_worker;             // k_post_lean: LDS bytes of one worker (no draw record)
    int qpar;                   // queue set of this step (0 unless bg)
    int spawn_slots;            // k_spawn workers
    int bg_tries;               // k_spawn: permutation attempts per job (until disjoint)
    int spawn_tries;            // in-step spawn-ahead jobs: permutation attempts per job (until disjoint)
    uint32_t spawn_gate;        // bg: k_spawn launches on this step's queue set so far (kQSpGen)
    int draw_wait;              // bg: 100 MHz ticks a reset waits for a record being drawn (claim_reset_mt)
    int spawn_delay;            // bg: 100 MHz ticks a k_spawn job sleeps once it marks a record DRAWING (tests)
    // lean encode (encode_lean): the frames copied into a zero-bordered LDS image
    // (lp columns / vr rows of padding, pw bytes per row, pframe bytes per frame)
    // so the crop needs no bounds test; unit -> (snake, row, col, frame) by
    // multiply-high reciprocals of ups = oh*ow*fs, rowl = ow*fs, fs, and of W/4
    int lean, lp, pw, pframe, lds_lean_bytes, ups, rowl;
    // table encode in k_post (encode_tbl_block; the lean geometry above, one
    // wave per env): its LDS carve -- the image at 0, window origins, patterns,
    // unit descriptors
    int tbl, tbl_base, tbl_pat, tbl_desc, lds_tbl_bytes;
    uint32_t mag_ups, mag_rowl, mag_fs, mag_wpr;
    // fused step (k_step, snake_kernels.hip): on, the logic groups, the step's
    // epoch, and word offsets into resetq of the logic-done counts, the groups'
    // done and claim flags, and the encodes' hand-off records (uint4 per env)
    int fused, nlg, fu_roles;
    uint32_t epoch;
    int64_t fu_ldone, fu_done, fu_claim, fu_hoff;
    double rf, rk, rl, rw, rt, max_steps;
};

int build_kcfg(const snake_cfg *c, int64_t num_envs, int64_t n_cand, KCfg *k);
int layout_of(const snake_cfg *c, int64_t num_envs, snake_layout *out);
// word offset in resetq of the fused step's area (after the two queue sets), and its words
int64_t fused_base(int64_t num_envs);
int64_t fused_words(int64_t num_envs);
void set_error(const char *fmt, ...);

// launchers (snake_kernels.hip)
int launch_seed(const KCfg &k, const snake_state &st, uint32_t base_seed, int64_t env_offset,
                void *stream);
int launch_reset(const KCfg &k, const snake_state &st, const uint8_t *mask, const snake_out &o,
                 void *stream);
int launch_step(const KCfg &k, const snake_state &st, const int8_t *actions, const snake_out &o,
                void *stream);
int wait_background(const snake_state &st, void *stream);
int release_background(const snake_state &st);
int launch_render(const KCfg &k, const snake_state &st, const uint8_t *palette, uint8_t *rgb,
                  void *stream);

}  // namespace snake
