// snake_capi.cpp -- C-ABI entry points (include/snake_env.h): config validation,
// buffer planning, the static spawn-pose table and argument checks before the
// HIP launches in snake_kernels.hip.
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <math.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

#include "snake_internal.h"

#ifndef SNAKE_SPAWN_PRIO_SMALL   // (A/B builds: scripts/build_variants.sh)
#define SNAKE_SPAWN_PRIO_SMALL 3
#endif

namespace snake {

static thread_local char g_err[512];

void set_error(const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
}

static int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

static int pow2_at_least(int x)
{
    int p = 1;
    while (p < x) p <<= 1;
    return p;
}

// SnakeEnv.__init__ argument rules (snake_env.py:58-129) plus this
// implementation's static limits (documented in DESIGN.md).
static int check_cfg(const snake_cfg *c)
{
    if (!c) { set_error("cfg is NULL"); return SNAKE_E_CONFIG; }
    if (c->height < 3 || c->height > 255 || c->width < 3 || c->width > 255) {
        set_error("height/width must be in [3, 255] (got %d x %d)", c->height, c->width);
        return SNAKE_E_CONFIG;
    }
    if (c->num_snakes < 1 || c->num_snakes > kMaxSnakes) {
        set_error("num_snakes must be in [1, %d] (got %d)", kMaxSnakes, c->num_snakes);
        return SNAKE_E_CONFIG;
    }
    if (c->snake_length < 2 || c->snake_length > 63) {
        // Snake.__init__ asserts len(coords) > 1 (core/snake.py:54)
        set_error("snake_length must be in [2, 63] (got %d)", c->snake_length);
        return SNAKE_E_CONFIG;
    }
    if (c->snake_length * c->num_snakes > kWave) {
        set_error("num_snakes * snake_length must be <= 64 (got %d)", c->snake_length * c->num_snakes);
        return SNAKE_E_CONFIG;
    }
    if (c->vision_range < 0 || 2 * c->vision_range + 1 > 255) {
        set_error("vision_range must be None/0 or in [1, 127] (got %d)", c->vision_range);
        return SNAKE_E_CONFIG;
    }
    if (c->frame_stack < 1 || c->frame_stack > 16) {
        set_error("frame_stack must be in [1, 16] (got %d)", c->frame_stack);
        return SNAKE_E_CONFIG;
    }
    if (c->observer != 0 && c->observer != 1) {
        set_error("observer must be 'snake' or 'human'");
        return SNAKE_E_CONFIG;
    }
    if (c->num_fruits < 1 || c->num_fruits > kMaxFruits) {
        // num_fruits == 0 makes the reference paint the whole grid FRUIT
        // (grid[None, None] = 2 at snake_env.py:147-148): not supported.
        set_error("num_fruits must be in [1, %d] (got %d)", kMaxFruits, c->num_fruits);
        return SNAKE_E_CONFIG;
    }
    int interior = (c->height - 2) * (c->width - 2);
    if (interior < c->num_snakes * c->snake_length + 1) {
        set_error("grid too small for %d snakes of length %d", c->num_snakes, c->snake_length);
        return SNAKE_E_CONFIG;
    }
    return SNAKE_OK;
}

// ---- spawn-pose table: dfs_sweep_empty(make_grid(H, W), L), grid_util.py:73-115.
// Paths are self-avoiding walks of L empty cells, head = first cell, extended in
// SHIFTS order (0,+1),(+1,0),(0,-1),(-1,0) (grid_util.py:7-11); a walk is kept only
// while its head has a free neighbour outside the walk (_head_blocked). Iterative
// DFS; emits int16 cell indices r*W+c.
struct Dfs {
    int H, W, L;
    std::vector<uint8_t> empty;
    std::vector<int16_t> *out;
    int64_t count = 0;
    int path[64];
    int dir_state[64];
};

static bool in_path(const Dfs &d, int n, int cell)
{
    for (int i = 0; i < n; i++)
        if (d.path[i] == cell) return true;
    return false;
}

static bool head_blocked(const Dfs &d, int n, int extra)
{
    static const int dr[4] = {0, 1, 0, -1}, dc[4] = {1, 0, -1, 0};
    int hr = d.path[0] / d.W, hc = d.path[0] % d.W, blocked = 0;
    for (int s = 0; s < 4; s++) {
        int r = hr + dr[s], c = hc + dc[s];
        int cell = r * d.W + c;
        if (r < 0 || c < 0 || r >= d.H || c >= d.W || !d.empty[cell] || in_path(d, n, cell) ||
            cell == extra)
            blocked++;
    }
    return blocked == 4;
}

static void dfs_from(Dfs &d, int start)
{
    static const int dr[4] = {0, 1, 0, -1}, dc[4] = {1, 0, -1, 0};
    int n = 1;
    d.path[0] = start;
    d.dir_state[0] = 0;
    if (d.L == 1) { d.count++; return; }
    while (n > 0) {
        if (n == d.L) {  // complete walk
            if (d.out) d.out->insert(d.out->end(), d.path, d.path + d.L);
            d.count++;
            n--;
            continue;
        }
        int &s = d.dir_state[n - 1];
        if (s >= 4) { n--; continue; }
        int cur = d.path[n - 1];
        int r = cur / d.W + dr[s], c = cur % d.W + dc[s];
        s++;
        if (r < 0 || c < 0 || r >= d.H || c >= d.W) continue;
        int cell = r * d.W + c;
        if (!d.empty[cell] || in_path(d, n, cell)) continue;
        if (head_blocked(d, n, cell)) continue;
        d.path[n] = cell;
        d.dir_state[n] = 0;
        n++;
    }
}

static int64_t build_table(int H, int W, int L, std::vector<int16_t> *out)
{
    Dfs d;
    d.H = H; d.W = W; d.L = L;
    d.empty.assign((size_t)H * W, 0);
    for (int r = 1; r < H - 1; r++)
        for (int c = 1; c < W - 1; c++) d.empty[(size_t)r * W + c] = 1;  // make_grid :14-20
    d.out = out;
    for (int cell = 0; cell < H * W; cell++)
        if (d.empty[cell]) dfs_from(d, cell);
    return d.count;
}

// Spawn-pose table per (H, W, L), memoised (snake_step/snake_reset re-plan on
// every call), and per S the probability that S poses drawn as
// permutation(n_cand)[:S] are pairwise disjoint (_generate_snakes' retry test,
// snake_env.py:576-589), estimated once by sampling.
struct PoseTable {
    int64_t n = 0;
    std::vector<int16_t> cells;
    std::map<int, std::pair<double, int64_t>> p_disjoint;   // S -> (estimate, samples)
};

static std::mutex g_table_mu;

static PoseTable &pose_table(int H, int W, int L)   // g_table_mu held
{
    static std::map<std::tuple<int, int, int>, PoseTable> memo;
    auto key = std::make_tuple(H, W, L);
    auto it = memo.find(key);
    if (it != memo.end()) return it->second;
    PoseTable t;
    t.n = build_table(H, W, L, &t.cells);
    return memo.emplace(key, std::move(t)).first->second;
}

static int64_t cached_count(int H, int W, int L)
{
    std::lock_guard<std::mutex> lock(g_table_mu);
    return pose_table(H, W, L).n;
}

// Monte-Carlo estimate (fixed seed, so deterministic) of P(S uniformly drawn
// distinct poses share no cell): up to 2e5 samples, stopping once 400 disjoint
// draws have been seen. *samples = the draws the estimate rests on.
static double disjoint_prob(int H, int W, int L, int S, int64_t *samples)
{
    std::lock_guard<std::mutex> lock(g_table_mu);
    PoseTable &t = pose_table(H, W, L);
    auto it = t.p_disjoint.find(S);
    if (it != t.p_disjoint.end()) {
        *samples = it->second.second;
        return it->second.first;
    }
    double p = 1.0;
    int64_t drawn = 0;
    if (S > 1 && t.n >= S) {
        std::vector<uint32_t> stamp((size_t)H * W, 0u);
        uint64_t x = 0x9e3779b97f4a7c15ull;
        auto next = [&x]() {
            x ^= x << 13; x ^= x >> 7; x ^= x << 17;
            return x;
        };
        int64_t hits = 0, m = 0;
        int64_t pick[kMaxSnakes];
        for (m = 1; m <= 200000 && hits < 400; m++) {
            bool ok = true;
            for (int k = 0; k < S; k++) {
                int64_t v;
                bool dup;
                do {
                    v = (int64_t)(next() % (uint64_t)t.n);
                    dup = false;
                    for (int j = 0; j < k; j++) dup |= pick[j] == v;
                } while (dup);
                pick[k] = v;
                for (int i = 0; i < L && ok; i++) {
                    uint32_t &c = stamp[t.cells[(size_t)v * L + i]];
                    ok = c != (uint32_t)m;
                    c = (uint32_t)m;
                }
            }
            hits += ok;
        }
        drawn = m - 1;
        p = (double)hits / (double)drawn;
    }
    t.p_disjoint[S] = std::make_pair(p, drawn);
    *samples = drawn;
    return p;
}

// Boards on which S disjoint spawn poses are this rare are rejected: a reset
// gives up after 2^16 permutations (snake_kernels.hip do_reset), which at this
// probability happens for fewer than ~2e-6 of the resets.
constexpr double kMinDisjoint = 2e-4;

// spawn-ahead threshold: by default envs with at most 3 live snakes
// (any env under coop, where one death ends the episode); -1 = off.  Measured
// r04h (same box, thr 2/3/4): cfg3 0.0853/0.0821/0.0900 ms, cfg4 0.0681/0.0636/
// 0.0635, cfg2 0.0478/0.0453/0.0451, cfg5 0.1141/0.1134/0.1136.
static int spawn_thr_of(const snake_cfg *c)
{
    int thr;
    if (c->spawn_ahead != 0) thr = c->spawn_ahead < 0 ? -1 : c->spawn_ahead;
    else thr = c->coop ? c->num_snakes : 3;
    if (c->autoreset != 1) thr = -1;   // (every-step resets: nothing to draw ahead)
    return thr;
}

// Background spawn-ahead (snake_kernels.hip k_spawn): the attempts leave the
// step entirely (the step never waits for them; two steps later its k_logic
// does, for the queue set). Needs spawn-ahead on (all-done auto-reset) and the
// draw record in LDS. cfg->spawn_background: 0 automatic, 1 on, -1 off.
// Automatic: boards of more than 8192 spawn poses, whose attempt outlasts a
// step (40x40: ~110 us), and small batches (<= 8192 envs, <= 64 MiB of
// observations per step), whose step is otherwise one in-step attempt's latency.
// Round 5 (one background stream per queue set, resets waiting for a record
// being drawn), same-box medians in ms: cfg2 (4096 envs) 0.0435 -> 0.0412, 1024
// envs 0.0404 -> 0.0340, cfg3 geometry at 8192 envs 0.0448 -> 0.0434; larger
// batches lose, the jobs slowing the concurrent encodes more than they save:
// cfg2 geometry at 8192 (100 MiB) 0.0460 -> 0.0512, cfg3 geometry at 16384
// 0.0495 -> 0.0539, cfg4 0.0580 -> 0.0672, cfg3 0.0838 -> 0.0887.
static bool bg_of(const snake_cfg *c, int64_t n_cand, int64_t N)
{
    const int64_t oh = c->vision_range ? 2 * c->vision_range + 1 : c->height;
    const int64_t ow = c->vision_range ? 2 * c->vision_range + 1 : c->width;
    const int64_t obs = N * c->num_snakes * oh * ow * 8 * c->frame_stack;
    const bool small = N <= 8192 && obs <= ((int64_t)64 << 20);
    const bool want = c->spawn_background != 0 ? c->spawn_background > 0 : (n_cand > 8192 || small);
    return want && spawn_thr_of(c) >= 0 && 2 * (n_cand + kWave) <= kJarrLdsMax;
}

// Lean-encode geometry (snake_kernels.hip encode_lean): the frames copied into a
// zero-bordered LDS image (lp columns / vr rows of padding, pw bytes per row,
// pframe bytes per frame) so the crop needs no bounds test; unit -> (snake, row,
// col, frame) by multiply-high reciprocals of ups = oh*ow*fs, rowl = ow*fs, fs,
// and of W/4. Used (lean = 1) for rings of 513 to 2 048 dwords, W % 4 == 0, when
// every reciprocal is exact: four-wave workgroups (cfg5 k_encode 91 -> 66 us);
// one wave per env measured slower beside the reset workers at one frame (cfg3
// step 0.1216 vs 0.1032 ms), so smaller rings keep the staged encode.
struct LeanGeom {
    int lean, lp, pw, pframe, lds_lean_bytes, ups, rowl;
    uint32_t mag_ups, mag_rowl, mag_fs, mag_wpr;
    int exact;   // every reciprocal exact, W % 4 == 0, an even unit count: the image and unit maps apply
};

static LeanGeom lean_geom(const snake_cfg *c)
{
    LeanGeom g;
    const int vr = c->vision_range, fs = c->frame_stack, H = c->height, W = c->width, S = c->num_snakes;
    const int oh = vr ? 2 * vr + 1 : H, ow = vr ? 2 * vr + 1 : W;
    const int64_t units = (int64_t)S * oh * ow * fs;
    g.lp = vr ? (int)round_up(vr, 4) : 0;
    g.pw = vr ? (int)round_up(W + g.lp + vr, 4) : W;
    g.pframe = (int)round_up((int64_t)(H + 2 * vr) * g.pw, 16);
    g.ups = oh * ow * fs;
    g.rowl = ow * fs;
    auto mag = [](uint64_t d) { return (uint32_t)(((1ull << 32) + d - 1) / d); };
    g.mag_ups = mag(g.ups); g.mag_rowl = mag(g.rowl); g.mag_fs = mag(fs);
    g.mag_wpr = mag(std::max(1, W / 4));
    g.lds_lean_bytes = (int)round_up((int64_t)fs * g.pframe, 16) + 4 * fs * kMaxSnakes;
    const int64_t fdw = (int64_t)fs * H * W / 4;
    bool ok = (units % 2) == 0 && units < (1 << 22) && W % 4 == 0;
    for (int64_t u = 0; ok && u < units; u++) {
        const int64_t q = ((uint64_t)u * g.mag_ups) >> 32, r0 = u - q * g.ups;
        const int64_t i = ((uint64_t)r0 * g.mag_rowl) >> 32, r1 = r0 - i * g.rowl;
        const int64_t j = fs == 1 ? r1 : ((uint64_t)r1 * g.mag_fs) >> 32;   // (snake_kernels.hip fdiv)
        ok = q == u / g.ups && i == r0 / g.rowl && j == r1 / fs;
    }
    for (int64_t x = 0; ok && x < (int64_t)H * W / 4; x++)
        ok = (W / 4 == 1 ? x : (int64_t)(((uint64_t)x * g.mag_wpr) >> 32)) == x / (W / 4);
    g.exact = ok ? 1 : 0;
    g.lean = ok && fdw > 8 * kWave && fdw <= 8 * 256 && g.lds_lean_bytes <= 48 * 1024 ? 1 : 0;
    return g;
}

// Queue entries per shard: k_logic's blocks of E envs spread over kQShards
// shards, room for every env of a shard's blocks.
static int64_t queue_cap(int64_t N, int64_t E)
{
    const int64_t blocks = (N + E - 1) / E;
    return (blocks + kQShards - 1) / kQShards * E;
}

// The fused step's area of resetq (snake_kernels.hip k_step), after the two
// queue sets: 64 logic-done counts (one line each), the groups' done and claim
// flags (at most N / 4 groups), the encodes' hand-off records (uint4 per env).
int64_t fused_base(int64_t N)
{
    const int64_t cap = std::max(queue_cap(N, 4), std::max(queue_cap(N, 8), queue_cap(N, 16)));
    return round_up(kQSets * (kNumQ * kQShards * cap + kQCounters), 4);
}
int64_t fused_words(int64_t N)
{
#ifdef SNAKE_NO_FUSED_AREA
    return 0 * N;
#endif
    return kQShards * kQSpread + 2 * round_up((N + 3) / 4, 4) + 4 * N;
}

int layout_of(const snake_cfg *c, int64_t N, snake_layout *o)
{
    int rc = check_cfg(c);
    if (rc) return rc;
    if (N < 1 || N > (int64_t)1 << 26) {
        set_error("num_envs must be in [1, 2^26] (got %lld)", (long long)N);
        return SNAKE_E_ARG;
    }
    memset(o, 0, sizeof *o);
    const int64_t S = c->num_snakes, fs = c->frame_stack, HW = (int64_t)c->height * c->width;
    const int oh = c->vision_range ? 2 * c->vision_range + 1 : c->height;
    const int ow = c->vision_range ? 2 * c->vision_range + 1 : c->width;
    o->grid_stride = (int32_t)round_up(HW, 16);
    // >= 16: the step reads the rings as aligned 8-byte chunks and writes 4-byte words
    o->ring_cap = std::max(16, pow2_at_least((c->height - 2) * (c->width - 2)));
    o->n_cand = cached_count(c->height, c->width, c->snake_length);
    o->obs_h = oh; o->obs_w = ow; o->obs_c = 8 * c->frame_stack;
    o->grid = N * fs * o->grid_stride;
    o->snake = N * S * 4 * 4;
    o->body = N * S * o->ring_cap;
    o->env = N * kEnvRec * 4;
    o->ctr = N * fs * S * 2;
    o->stats = N * S * (int64_t)sizeof(snake_epi_stat);
    o->mt = N * kMtN * 4;
    o->cand = o->n_cand * c->snake_length * 2;
    // What the reset workers record of a permutation (snake_kernels.hip
    // perm_trace): the u16 draw record in LDS up to kJarrLdsMax bytes, else one
    // global u32 link table per reset worker.
    const int64_t link = (round_up(o->n_cand, 4) + kWave) * 4;
    // (also the four-wave lean-encode boards' auto-resets: k_post_lean's workers
    // keep no draw record in LDS)
    const bool lean_workers = c->autoreset == 1 && lean_geom(c).lean;
    o->jscratch = (round_up(2 * (o->n_cand + kWave), 16) <= kJarrLdsMax && !lean_workers)
                      ? 0 : std::min<int64_t>(N, kResetSlots) * link;
    // (background spawn-ahead: one record per queue set and env, see k_spawn)
    o->spawn = (bg_of(c, o->n_cand, N) ? kQSets : 1) * N * kSpawnStride * 4;
    {   // auto-reset and spawn-ahead queues: kQShards shards each (k_logic block %
        // kQShards) with room for every env of its blocks, + the step's counters
        // (kQCount, each in its own line); sized for any k_logic lane grouping
        // + the fused step's flags, counts and hand-off records
        o->resetq = (fused_base(N) + fused_words(N)) * 4;
    }
    o->obs = N * S * oh * ow * 8 * fs;
    o->rew = N * S * 8;
    o->done = N * S;
    o->ep_done = N;
    o->rank = N * S * 4;
    o->ep_stats = N * 4 * S * 8;
    o->err = N * 4;
    if (o->n_cand > 65535) {
        set_error("%lld spawn poses: more than the 65535 the reset scratch indexes",
                  (long long)o->n_cand);
        return SNAKE_E_CONFIG;
    }
    if (o->n_cand < S) {
        set_error("only %lld spawn poses for %lld snakes", (long long)o->n_cand, (long long)S);
        return SNAKE_E_CONFIG;
    }
    int64_t samples = 0;
    const double pd = disjoint_prob(c->height, c->width, c->snake_length, (int)S, &samples);
    if (pd < kMinDisjoint) {
        set_error("%dx%d board too crowded: %lld snakes of length %d are disjoint in only "
                  "%.2g of the spawn draws (Monte-Carlo estimate: %lld of %lld sampled draws; the limit is %.0e; "
                  "the reference would retry ~%.0f permutations per reset)",
                  c->height, c->width, (long long)S, c->snake_length, pd, (long long)llround(pd * samples),
                  (long long)samples, kMinDisjoint, pd > 0 ? 1.0 / pd : 1e30);
        return SNAKE_E_CONFIG;
    }
    return SNAKE_OK;
}

int build_kcfg(const snake_cfg *c, int64_t N, int64_t n_cand, KCfg *k)
{
    snake_layout lay;
    int rc = layout_of(c, N, &lay);
    if (rc) return rc;
    if (n_cand != lay.n_cand) {
        set_error("spawn-pose table has %lld rows, expected %lld", (long long)n_cand,
                  (long long)lay.n_cand);
        return SNAKE_E_ARG;
    }
    memset(k, 0, sizeof *k);
    k->N = (int)N;
    k->H = c->height; k->W = c->width; k->HW = c->height * c->width;
    k->S = c->num_snakes; k->L = c->snake_length; k->vr = c->vision_range;
    k->fs = c->frame_stack; k->observer = c->observer; k->num_fruits = c->num_fruits;
    k->coop = c->coop ? 1 : 0; k->autoreset = c->autoreset == 2 ? 2 : (c->autoreset ? 1 : 0);
    k->oh = lay.obs_h; k->ow = lay.obs_w;
    k->units = k->S * k->oh * k->ow * k->fs;
    k->grid_stride = lay.grid_stride; k->ring_cap = lay.ring_cap; k->n_cand = (int)lay.n_cand;
    k->cs = (k->HW + kWave - 1) / kWave;
    k->ring_bytes = k->fs * k->grid_stride;
    // 128 units in mixed radix (f: fs, j: ow, i: oh, k: S)
    int64_t a = 128;
    k->adv_f = (int)(a % k->fs); a /= k->fs;
    k->adv_j = (int)(a % k->ow); a /= k->ow;
    k->adv_i = (int)(a % k->oh); a /= k->oh;
    k->adv_k = (int)a;
    int off = 0;
    k->lds_frames = off; off += (int)round_up((int64_t)k->fs * k->grid_stride, 16);
    k->lds_centers = off; off += (int)round_up(4 * k->fs * kMaxSnakes, 16);
    k->lds_fruit = off; off += (int)round_up(2 * kMaxFruits, 16);
    {   // staged encode: whole snakes per group, every group start 16-byte aligned
        const int64_t P = (int64_t)k->oh * k->ow * 8 * k->fs;       // obs bytes per snake
        int g = 0;
        if ((int64_t)k->S * P <= kStageMax) {
            g = k->S;
        } else {
            g = (int)std::min<int64_t>(k->S, kStageMax / P);
            if (P % 16 != 0) g &= ~1;
        }
        k->enc_group = g;
        k->lds_stage = off;
        k->lds_worker = off;   // (frames, centres, fruit buffer: a resets-only worker without the draw record)
        if (g > 0) off += (int)round_up(g * P, 16);
        const uint64_t fsoh = (uint64_t)k->fs * k->oh, oh = (uint64_t)k->oh;
        k->mag_fsoh = (uint32_t)(((1ull << 32) + fsoh - 1) / fsoh);
        k->mag_oh = (uint32_t)(((1ull << 32) + oh - 1) / oh);
        k->mag_W = (uint32_t)(((1ull << 32) + k->W - 1) / k->W);
        const uint64_t n16 = (uint64_t)k->grid_stride / 16;
        k->mag_n16 = (uint32_t)(((1ull << 32) + n16 - 1) / n16);
    }
    k->link_stride = (int)round_up(k->n_cand, 4) + kWave;
    // the LDS draw record: u16 per index < n_cand + one dummy slot per lane
    int jbytes = (int)round_up(2 * ((int64_t)k->n_cand + kWave), 16);
    k->link_in_lds = jbytes <= kJarrLdsMax;
    // up to 32 768 envs the attempts' chain sets the shared phase: their link
    // table as u32 in LDS (ds_min while drawing, then a pointer chase of ~ln n
    // hops instead of scanning the u16 record: ~15 K of ~60 K cycles per
    // attempt) -- cfg2 0.0451 -> 0.0430 ms, cfg4 0.0627 -> 0.0602; at 65 536
    // envs the doubled LDS costs the encodes their occupancy (cfg3 0.0842 ->
    // 0.0994), so there the u16 record stays
    if (k->link_in_lds && N <= 32768 && !bg_of(c, n_cand, N) && 4 * (int64_t)k->link_stride <= kJarrLdsMax) {
        k->link32 = 1;
        jbytes = 4 * k->link_stride;
    }
    // reset workers (<= kResetSlots, the global link tables are sized for that)
    k->reset_slots = (int)std::min<int64_t>(N, kResetSlots);
    const bool bg = bg_of(c, n_cand, N);
    // small boards with the background kernel: the workers only paint resets
    // from records (≈65 per step at cfg2), so 512 of them (same box, ms per
    // step: cfg2 0.0399 -> 0.0394 and 0.0401 -> 0.0397; 256: 0.0397; 40x40
    // boards within noise at 256-1024, kept at 2 048)
    const bool bg_small = bg && n_cand <= 8192 && N <= 8192;   // (not a forced background kernel on a big batch)
    if (bg_small) k->reset_slots = (int)std::min<int64_t>(N, 512);
    // spawn-ahead jobs at 1, below the encodes; small batches with in-step
    // spawn-ahead higher (a lone attempt is there the step's critical path:
    // cfg2 0.0510 -> 0.0494 ms; at cfg3 it costs 0.0905 -> 0.0960). Until round
    // 5 the workers mapped every value >= 2 to s_setprio 2, the encodes' level
    // (ADVICE r4): round 4's "priority 3" (cfg4 0.0595 -> 0.0584 ms) ran at 2.
    k->spawn_prio = N <= 32768 && !bg ? SNAKE_SPAWN_PRIO_SMALL : 1;
    // the encodes above the spawn-ahead jobs: the bandwidth-bound encodes then
    // keep HBM busy while the compute-bound workers fill the issue gaps (cfg3
    // 0.1275 -> 0.1200 ms against the hardware default 0). With background
    // spawn-ahead the step's resets are the critical path beside the encodes
    // instead: 0 (cfg5 0.160 -> 0.135 ms).
    k->encode_prio = bg ? 0 : 2;   // (2 on small background boards: cfg2 0.0399 -> 0.0403)
    {
        // k_logic's lanes per env (4, 8 or 16 >= S; 64 / that = envs per wave):
        // the fewest lanes that hold S snakes; small batches at least 8 (more,
        // shorter waves: cfg2's 4 096 envs k_logic 16.4 -> 15.3 us, step 0.0540
        // -> 0.0527 ms; 16 lanes 18.0 us; at cfg3 8 lanes cost 6 us)
        const int ms_min = k->S <= 4 ? 4 : (k->S <= 8 ? 8 : 16);
        k->logic_ms = N <= 8192 ? std::max(ms_min, 8) : ms_min;   // (round 5, background cfg2: 4 lanes 0.0403 vs 0.0399)
    }
    // k_logic's LDS carve (snake_kernels.hip k_logic) per wave: E frames, the
    // fruit buffer, the respawn raws and cells
    auto logic_lds = [&](int G) {
        const int E = kWave / G;
        return (int)round_up((int64_t)E * k->grid_stride + 2 * kMaxFruits + E * G * 4 * 4 + E * G * 2, 16);   // (kRespawnT = 4)
    };
    // large boards: fewer envs per wave until one wave's frames fit a workgroup
    while (k->logic_ms < 16 && logic_lds(k->logic_ms) > kLdsLimit) k->logic_ms *= 2;
    k->lds_logic = logic_lds(k->logic_ms);
    if (k->lds_logic > kLdsLimit) {
        set_error("%dx%d board: k_logic's %d frames per wave (%d bytes) do not fit the %d-byte LDS", k->H, k->W,
                  kWave / k->logic_ms, k->lds_logic, kLdsLimit);
        return SNAKE_E_CONFIG;
    }
    // four independent waves per workgroup where their LDS fits (round 4: k_logic
    // cfg4 20.4 -> 19.4 us, cfg5 21.9 -> 21.1 against one), else one
    k->logic_wpb = 4 * (int64_t)k->lds_logic <= kLdsLimit ? 4 : 1;
    k->q_envs_per_block = kWave / k->logic_ms;
    k->q_cap = (int)queue_cap(N, k->q_envs_per_block);
    k->spawn_thr = spawn_thr_of(c);
    // small batches with the background kernel: the attempts leave the step and
    // the CUs have room, so one live snake more (round 5, same box, ms per step,
    // threshold 3 -> 4: cfg2 0.0409 -> 0.0403, cfg3 geometry at 8 192 envs
    // 0.0434 -> 0.0425; 40x40 boards unchanged at 3: cfg5 0.0826 vs 0.0827)
    if (bg_small && c->spawn_ahead == 0 && !c->coop && k->spawn_thr == 3) k->spawn_thr = 4;
    k->bg = bg ? 1 : 0;
    // k_spawn workers: 512 on small background boards (≈130 jobs per step at
    // cfg2: 0.0397 -> 0.0391 ms, same box; 256: 0.0392), 2 048 on 40x40 (cfg5:
    // 512 0.0827-0.0832, 1 024 0.0822, 2 048 0.0823)
    k->spawn_slots = (int)std::min<int64_t>(N, bg_small ? 512 : kResetSlots);
#ifndef SNAKE_BG_TRIES_SMALL
#define SNAKE_BG_TRIES_SMALL 2
#endif
    // k_spawn: attempts per job. Two on small background boards since the four
    // queue sets (round 6, same box, ms per step: cfg2 0.0397 -> 0.0380, cfg3s8
    // 0.0414 -> 0.0401; four tries slower, profiles/r06_ab_qsets.txt); one on
    // 40x40 (4 measured 0.30 ms at cfg5: the kernel then gates k_logic)
    k->bg_tries = bg_small ? SNAKE_BG_TRIES_SMALL : 1;
    k->spawn_tries = 1;   // attempts per in-step spawn-ahead job (2 measured cfg3 0.0875 -> 0.103 ms: a retry doubles the chain)
    k->lds_obs_bytes = off;
    {
        const LeanGeom g = lean_geom(c);
        k->lean = g.lean; k->lp = g.lp; k->pw = g.pw; k->pframe = g.pframe;
        k->lds_lean_bytes = g.lds_lean_bytes; k->ups = g.ups; k->rowl = g.rowl;
        k->mag_ups = g.mag_ups; k->mag_rowl = g.mag_rowl; k->mag_fs = g.mag_fs; k->mag_wpr = g.mag_wpr;
        // the table encode (snake_kernels.hip encode_tbl_block) where k_post runs
        // the encodes: rings of at most 512 dwords, the lean geometry exact
        const int64_t fdw = (int64_t)k->fs * k->HW / 4;
        int t = 0;
        k->tbl_base = (int)round_up((int64_t)k->fs * k->pframe, 16); t = k->tbl_base + 8 * k->fs * kMaxSnakes;
        k->tbl_pat = t; t += 8 * k->S * 160;   // (kPatV)
        k->tbl_desc = t; t += (int)round_up(4 * (int64_t)k->units, 16);
        k->lds_tbl_bytes = t;
        k->tbl = g.exact && !g.lean && fdw <= 8 * kWave && t <= 40 * 1024 ? 1 : 0;
        // also in k_post_lean's four-wave workgroups (tables shared by the
        // workgroup, two envs each): cfg5 0.1023-0.1031 -> 0.1013-0.1015 ms; four
        // or eight envs per workgroup 0.107 / 0.111
        if (g.lean && t <= 48 * 1024) k->tbl = 1;
    }
    // envs per encode wave (k_post's encodes: the next env's ring prefetched into
    // registers, at most 8 16-byte chunks per lane): two at 16 384 envs and more
    // (cfg3 0.1033 -> 0.0998 ms; 4, 8, 16, 32 measured 0.1016, 0.106, 0.114,
    // 0.135), one below (cfg2 0.0622 vs 0.0625); the lean encode two per workgroup
    k->enc_per_wave = k->lean ? 2 : (N >= 16384 && k->ring_bytes <= 8 * 1024 ? 2 : 1);
    if (k->tbl) k->enc_per_wave = k->lean ? 2 : 4;   // (the tables are built once per wave; 8 measured slower at cfg3)
    // (k_logic encoding the observations of its envs itself, from its LDS frames,
    // measured slower: cfg3 k_logic 24.8 -> 83.9 us against k_post 66.9 -> 57.6)
    // the reset workers never use the encode staging buffer: the draw record
    // overlays it (the workers' LDS is what k_encode's waves share the CUs with)
    k->lds_link = k->lds_stage;
    k->lds_bytes = k->link_in_lds ? std::max(off, k->lds_stage + jbytes) : off;
    if (k->lds_bytes > 64 * 1024) {
        set_error("grid ring of %d bytes per env does not fit the LDS budget", k->ring_bytes);
        return SNAKE_E_CONFIG;
    }
    {   // the fused step (snake_kernels.hip k_step): all-done auto-reset in the step
        // with the one-wave table encode (4 envs per wave), one frame and at most
        // 4 snakes (the hand-off record's crop centres), in-step spawn-ahead
        const int E = kWave / k->logic_ms;
        k->nlg = (int)((N + E - 1) / E);
        k->fused = c->autoreset == 1 && k->tbl && !k->lean && !k->bg && k->fs == 1 && k->S <= 4 &&
                   k->enc_per_wave == 4 && E % 4 == 0 && (k->link32 || k->link_in_lds) ? 1 : 0;
        const int64_t fb = fused_base(N), groups = round_up((N + 3) / 4, 4);
        k->fu_ldone = fb;
        k->fu_done = fb + kQShards * kQSpread;
        k->fu_claim = k->fu_done + groups;
        k->fu_hoff = k->fu_claim + groups;
        k->epoch = 0;
    }
    k->rf = c->rew_fruit; k->rk = c->rew_kill; k->rl = c->rew_lose; k->rw = c->rew_win;
    k->rt = c->rew_time; k->max_steps = c->max_episode_steps;
    return SNAKE_OK;
}

static int check_state(const KCfg &k, const snake_state *st, bool need_all)
{
    if (!st || !st->grid || !st->snake || !st->body || !st->env || !st->ctr || !st->stats ||
        !st->mt || !st->cand) {
        set_error("snake_state has a NULL buffer");
        return SNAKE_E_ARG;
    }
    if (!st->resetq || !st->spawn) {
        set_error("snake_state.resetq / spawn is NULL");
        return SNAKE_E_ARG;
    }
    if ((!k.link_in_lds || (k.lean && k.autoreset == 1)) && !st->jscratch) {
        set_error("snake_state.jscratch is required for this config (n_cand=%d)", k.n_cand);
        return SNAKE_E_ARG;
    }
    (void)need_all;
    return SNAKE_OK;
}

static int check_out(const snake_out *o, bool step)
{
    if (!o || !o->obs) { set_error("snake_out.obs is NULL"); return SNAKE_E_ARG; }
    if (step && (!o->rew || !o->done || !o->ep_done || !o->rank || !o->ep_stats || !o->err)) {
        set_error("snake_out has a NULL step buffer");
        return SNAKE_E_ARG;
    }
    return SNAKE_OK;
}

static int64_t n_cand_of(const snake_cfg *c)
{
    snake_layout lay;
    if (layout_of(c, 1, &lay)) return -1;
    return lay.n_cand;
}

// build_kcfg of the step/reset/seed calls, memoised per thread: the plan is a
// pure function of (cfg, num_envs) (the environment knobs are read once), and
// re-planning on every snake_step cost host time on the step's critical path
// at small N (layout_of twice, two mutex-guarded table lookups).
static int plan_cached(const snake_cfg *c, int64_t N, KCfg *k)
{
    struct Entry {
        snake_cfg cfg;
        int64_t n;
        KCfg k;
    };
    thread_local Entry memo[8];
    thread_local int used = 0, next = 0;
    if (!c) { set_error("cfg is NULL"); return SNAKE_E_CONFIG; }
    for (int i = 0; i < used; i++) {
        if (memo[i].n == N && memcmp(&memo[i].cfg, c, sizeof *c) == 0) {
            *k = memo[i].k;
            return SNAKE_OK;
        }
    }
    int rc = build_kcfg(c, N, n_cand_of(c), k);
    if (rc) return rc;
    Entry &e = memo[next];
    e.cfg = *c;
    e.n = N;
    e.k = *k;
    next = (next + 1) % 8;
    used = used < 8 ? used + 1 : 8;
    return SNAKE_OK;
}

}  // namespace snake

using namespace snake;

extern "C" {

int snake_abi_version(void) { return SNAKE_ABI_VERSION; }

const char *snake_last_error(void) { return g_err; }

int snake_plan(const snake_cfg *cfg, int64_t num_envs, snake_layout *out)
{
    if (!out) { set_error("out is NULL"); return SNAKE_E_ARG; }
    g_err[0] = 0;
    int rc = layout_of(cfg, num_envs, out);
    if (rc) return rc;
    // (and every launch-side limit: a config the step cannot launch fails here)
    KCfg k;
    return build_kcfg(cfg, num_envs, out->n_cand, &k);
}

int64_t snake_build_candidates(const snake_cfg *cfg, int16_t *host_out, int64_t capacity)
{
    int rc = check_cfg(cfg);
    if (rc) return rc;
    std::vector<int16_t> v;
    int64_t n = build_table(cfg->height, cfg->width, cfg->snake_length, &v);
    if (host_out) {
        if (capacity < (int64_t)v.size()) {
            set_error("capacity %lld < %lld table entries", (long long)capacity, (long long)v.size());
            return SNAKE_E_ARG;
        }
        memcpy(host_out, v.data(), v.size() * sizeof(int16_t));
    }
    return n;
}

int snake_seed(const snake_cfg *cfg, const snake_state *st, int64_t num_envs, uint32_t base_seed,
               int64_t env_offset, void *stream)
{
    KCfg k;
    int rc = plan_cached(cfg, num_envs, &k);
    if (rc) return rc;
    if ((rc = check_state(k, st, false))) return rc;
    if (env_offset < 0) { set_error("env_offset < 0"); return SNAKE_E_ARG; }
    return launch_seed(k, *st, base_seed, env_offset, stream);
}

int snake_reset(const snake_cfg *cfg, const snake_state *st, int64_t num_envs,
                const uint8_t *env_mask, const snake_out *out, void *stream)
{
    KCfg k;
    int rc = plan_cached(cfg, num_envs, &k);
    if (rc) return rc;
    if ((rc = check_state(k, st, true))) return rc;
    if ((rc = check_out(out, false))) return rc;
    return launch_reset(k, *st, env_mask, *out, stream);
}

int snake_sync(const snake_cfg *cfg, const snake_state *st, int64_t num_envs, void *stream)
{
    KCfg k;
    int rc = plan_cached(cfg, num_envs, &k);
    if (rc) return rc;
    if (!st || !st->env) { set_error("snake_state.env is NULL"); return SNAKE_E_ARG; }
    return wait_background(*st, stream);
}

int snake_step(const snake_cfg *cfg, const snake_state *st, int64_t num_envs, const int8_t *actions,
               const snake_out *out, void *stream)
{
    KCfg k;
    int rc = plan_cached(cfg, num_envs, &k);
    if (rc) return rc;
    if ((rc = check_state(k, st, true))) return rc;
    if ((rc = check_out(out, true))) return rc;
    if (!actions) { set_error("actions is NULL"); return SNAKE_E_ARG; }
    return launch_step(k, *st, actions, *out, stream);
}

int snake_release(const snake_cfg *cfg, const snake_state *st, int64_t num_envs)
{
    KCfg k;
    int rc = plan_cached(cfg, num_envs, &k);
    if (rc) return rc;
    if (!st || !st->env) { set_error("snake_state.env is NULL"); return SNAKE_E_ARG; }
    return release_background(*st);
}

int snake_render_rgb(const snake_cfg *cfg, const snake_state *st, int64_t num_envs,
                     const uint8_t *palette, uint8_t *rgb, void *stream)
{
    KCfg k;
    int rc = plan_cached(cfg, num_envs, &k);
    if (rc) return rc;
    if (!st || !st->grid || !st->env) { set_error("snake_state.grid/env is NULL"); return SNAKE_E_ARG; }
    if (!palette) { set_error("palette is NULL"); return SNAKE_E_ARG; }
    if (!rgb) { set_error("rgb is NULL"); return SNAKE_E_ARG; }
    return launch_render(k, *st, palette, rgb, stream);
}

}  // extern "C"
