/*
 * snake_env.h -- C-ABI of the MI355X-native batched multi-snake environment.
 *
 * The drop-in boundary for the reference's hot path (tranthai189765/MARL-Snake,
 * marlenv/marlenv/envs/snake_env.py SnakeEnv.reset/step, reached through
 * marlenv/marlenv/wrappers.py make_snake). The reference is pure Python, so its
 * "FFI" for this path is the Python method surface; the product's Python host
 * layer (marl-snake_amd/marlenv) binds these entry points with ctypes
 * (marl-snake_amd/marlenv/_native.py) and re-exposes make_snake()/reset()/step().
 *
 * Conventions
 *   - plain C types only; every buffer pointer is DEVICE memory allocated and
 *     owned by the caller (PyTorch); the library allocates nothing on the device.
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream); calls
 *     are stream-ordered and asynchronous; not re-entrant per state.
 *   - return 0 on success, a negative SNAKE_E* code on a bad argument (message in
 *     snake_last_error()), never abort.
 *   - env i of a batch is a standalone reference SnakeEnv after
 *     np.random.seed(base_seed + env_offset + i).
 */
#ifndef SNAKE_ENV_H
#define SNAKE_ENV_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SNAKE_ABI_VERSION 17

#define SNAKE_OK           0
#define SNAKE_E_CONFIG    -1   /* invalid snake_cfg (message says which field) */
#define SNAKE_E_ARG       -2   /* NULL / mis-sized buffer, num_envs out of range */
#define SNAKE_E_LAUNCH    -3   /* HIP launch error (message has hipGetErrorString) */

/* Environment configuration. Mirrors SnakeEnv.__init__ kwargs
 * (snake_env.py:58-129) and the gym ids of envs/__init__.py:3-16. */
typedef struct {
    int32_t height, width;      /* grid incl. walls, 3..255 */
    int32_t num_snakes;         /* S, 1..16 */
    int32_t snake_length;       /* initial length L >= 2 */
    int32_t vision_range;       /* 0 == None (full-map obs), else crop (2vr+1)^2 */
    int32_t frame_stack;        /* fs >= 1, obs channels = 8*fs */
    int32_t observer;           /* 0 = 'snake' (actions 0/1/2), 1 = 'human' (0..4) */
    int32_t num_fruits;         /* 1..64; default round(0.8*S) (:87-88) */
    double  rew_fruit, rew_kill, rew_lose, rew_win, rew_time;   /* reward_dict */
    double  max_episode_steps;  /* 1e4 by default (:56) */
    int32_t coop;               /* 1 = SnakeCoop-v1: episode ends when ANY snake dies */
    int32_t autoreset;          /* 1 = reset an env inside snake_step when all its dones
                                   are True and return the reset obs (vector-env semantics,
                                   wrappers.py:139-145); 0 = return the terminal obs;
                                   2 = reset every env after every step (gym 0.23.1's
                                   worker behind make_snake, wrappers.py:212) */
    int32_t spawn_ahead;        /* spawn-ahead threshold (snake_step): 0 = default (at most
                                   3 live snakes, 4 on small background batches of at most
                                   8192 spawn poses, every env under coop), -1 = off, k >= 1 =
                                   envs with at most k live snakes. Never changes results. */
    int32_t spawn_background;   /* 1 = the spawn-ahead attempts run in a background kernel on a
                                   stream of the library's (two per state) that outlives snake_step (see
                                   snake_sync, snake_release), 0 = automatic (on for boards of
                                   more than 8192 spawn poses, e.g. 40x40, and for batches of
                                   at most 8192 envs and 64 MiB of observations per step),
                                   -1 = off (inside the step). Needs spawn-ahead on and a draw record that fits LDS
                                   (at most 18 368 spawn poses). Never changes results. */
} snake_cfg;

/* Byte sizes of every caller-allocated buffer for num_envs envs (snake_plan). */
typedef struct {
    int64_t grid;       /* uint8  [N][fs][grid_stride]   grid ring (newest = env[2]) */
    int64_t snake;      /* int32  [N][S][4]              packed snake records: head/tail cells; heading,
                                                         alive, pending ring-word directions; ring head and
                                                         length; tail-direction queue (see k_logic) */
    int64_t body;       /* uint8  [N][S][ring_cap]       direction deques (rings), ring_cap >= 16 */
    int64_t env;        /* int32  [N][8]                 alive_snakes, episode_length, cur, mt_pos
                                                         (> 624: the key's twist is pending, position
                                                         624 + j = word j of the next key),
                                                         spawn-ahead status word (bits 0-1: 0 none,
                                                         1 partial, 2 ready, 3 being drawn by a background
                                                         job; bits 2-3: which of the env's four
                                                         records holds it (background spawn-ahead, one per
                                                         queue set); bits 4-31: the record's generation),
                                                         spawn failure (1: the last reset gave up, below);
                                                         words 6-7 unused */
    int64_t ctr;        /* uint16 [N][fs][S]             crop centre (r<<8|c) of each grid ring slot */
    int64_t stats;      /* snake_epi_stat [N][S]         running episode score/steps/fruits/kills */
    int64_t mt;         /* uint32 [N][624]               per-env MT19937 key */
    int64_t cand;       /* int16  [n_cand][L]            spawn-pose table (cell indices) */
    int64_t jscratch;   /* uint32 [min(N,2048)][round4(n_cand)+64] reset link tables, 0 when the
                                                         u16 draw record fits LDS (2*n_cand <= 36 KB)
                                                         and the board's auto-resets do not run beside
                                                         four-wave lean encodes (k_post_lean) */
    int64_t spawn;      /* uint32 [N][672]               spawn-ahead record: MT key, MT pos and the
                                                         S*L spawn cells (u16) of the env's next reset
                                                         ([4][N][672] with background spawn-ahead) */
    int64_t resetq;     /* int32  4 x ([3][64][cap] + [227*32]) sharded auto-reset and spawn-ahead
                                                         queues + the step's counters, one per 128-B
                                                         line; four sets, by step count mod 4; then the
                                                         fused step's flags and hand-off records
                                                         (zero-initialised) */
    int64_t obs;        /* uint8  [N][S][h][w][8*fs]     NHWC observations */
    int64_t rew;        /* double [N][S] */
    int64_t done;       /* uint8  [N][S] */
    int64_t ep_done;    /* uint8  [N]                    1 when the step ended the episode */
    int64_t rank;       /* int32  [N][S]                 info['rank'] where ep_done (elsewhere not written) */
    int64_t ep_stats;   /* double [N][4][S]              info episode_* where ep_done (elsewhere not written) */
    int64_t err;        /* int32  [N]                    1 = invalid action (reference KeyError: the
                                                         env is left unchanged, its rew/done are 0);
                                                         2 = its auto-reset gave up (below) */
    int64_t n_cand;     /* rows of the spawn-pose table */
    int32_t obs_h, obs_w, obs_c;
    int32_t grid_stride, ring_cap;
} snake_layout;

/* Running episode statistics of one snake (_reset_epi_stats, snake_env.py:
 * 385-389, 438-442): the score in float64 as the reference sums it; steps,
 * fruits and kills are the reference's integer-valued float64 sums held as
 * integers (fruits < 65536: a snake's length is bounded by the board; kills
 * <= num_snakes: every kill credit is a death in the episode). */
typedef struct {
    double   score;
    uint32_t steps;
    uint16_t fruits, kills;
} snake_epi_stat;

typedef struct {        /* device state buffers (layouts in snake_layout) */
    uint8_t  *grid;
    int32_t  *snake;
    uint8_t  *body;
    int32_t  *env;
    uint16_t *ctr;
    snake_epi_stat *stats;
    uint32_t *mt;
    const int16_t *cand;
    uint32_t *jscratch; /* may be NULL when layout.jscratch == 0 */
    uint32_t *spawn;
    int32_t  *resetq;   /* zero-initialised once by the caller */
} snake_state;

typedef struct {        /* device output buffers of one step/reset */
    uint8_t *obs;
    double  *rew;
    uint8_t *done;
    uint8_t *ep_done;
    int32_t *rank;
    double  *ep_stats;
    int32_t *err;
} snake_out;

/* Validate cfg and compute buffer sizes. Replaces SnakeEnv.__init__'s checks and
 * observation_space shape (snake_env.py:58-129). Also rejects boards on which S
 * random spawn poses are disjoint in fewer than 2e-4 of the draws (estimated by
 * sampling): the reference's _generate_snakes retries forever (:576-589), a reset
 * here gives up after 2^16 permutations -- sets env word 5 (and err = 2 for an
 * auto-reset) -- which the bound keeps below ~2e-6 per reset. */
int snake_plan(const snake_cfg *cfg, int64_t num_envs, snake_layout *out);

/* Host-side spawn-pose table = dfs_sweep_empty(make_grid(H, W), L) in reference
 * order (grid_util.py:73-115), as int16 cell indices r*W+c, n_cand x L. Static per
 * (H, W, L): computed once, uploaded once. Returns n_cand, or < 0. */
int64_t snake_build_candidates(const snake_cfg *cfg, int16_t *host_out, int64_t capacity);

/* Seed env i's MT19937 with base_seed + env_offset + i (np.random.seed,
 * snake_env.py:581 / grid_util.py:130 use the global legacy RandomState). */
int snake_seed(const snake_cfg *cfg, const snake_state *st, int64_t num_envs,
               uint32_t base_seed, int64_t env_offset, void *stream);

/* SnakeEnv.reset() (snake_env.py:131-159) for every env whose env_mask byte is
 * nonzero (env_mask == NULL: all envs); writes out->obs for those envs. With
 * spawn-ahead on (autoreset on all-done, cfg->spawn_ahead != -1) each reset env
 * also gets the spawn poses of its NEXT reset drawn into its spawn record (up to
 * 4 permutation attempts: status ready, else partial), see snake_step. */
int snake_reset(const snake_cfg *cfg, const snake_state *st, int64_t num_envs,
                const uint8_t *env_mask, const snake_out *out, void *stream);

/* SnakeEnv.step(actions) (snake_env.py:301-414) for all envs at once; actions is
 * int8 [N][S]. With cfg->autoreset an env whose dones are all True is reset in
 * the same call and its out->obs holds the reset observation. Launches, all on
 * `stream`: k_logic (the game rules of every env, queueing the auto-resets),
 * then k_post, whose first blocks are the reset workers and the rest the encodes
 * of every other env's observation (k_post_lean: four workers per workgroup, then
 * four-wave lean encodes, for boards with rings of 513-2048 dwords such as 40x40
 * with 4 frames). Background spawn-ahead adds k_spawn on the library's stream
 * for the state (snake_sync). Without autoreset: k_logic, k_encode; every-step
 * autoreset: k_logic, k_autoreset, k_encode.
 *
 * Spawn-ahead: a reset's spawn poses depend only on the env's MT19937 state, which
 * changes only at fruit respawns and resets. With autoreset, k_logic also queues
 * every env that is close to the end of its episode (at most 2 snakes alive, or
 * any env under coop) and has no ready record for its current MT state, and the
 * k_autoreset workers, after the step's resets, run one permutation attempt of
 * that env's NEXT reset into its spawn record (st->spawn). A later reset of the
 * env starts from the record (MT key, position, poses) when no draw has touched
 * the MT state since; a fruit respawn or a reset invalidates it. Results are
 * identical with or without it (it only moves draws off the step's critical
 * path); cfg->spawn_ahead = -1 disables it. A caller that
 * rewrites an env's MT key or position itself must zero that env's status word
 * (env word 4), after snake_sync. */
int snake_step(const snake_cfg *cfg, const snake_state *st, int64_t num_envs,
               const int8_t *actions, const snake_out *out, void *stream);

/* With background spawn-ahead (cfg->spawn_background) a spawn kernel of the
 * last snake_step may still be running when the call returns; it writes only
 * st->spawn and env word 4, and the next snake_step / snake_reset / snake_seed
 * order themselves after it. Before the caller reads or writes the state
 * buffers itself (snapshots, set_mt_state, freeing them), snake_sync makes
 * `stream` wait for it (a no-op without background work). */
int snake_sync(const snake_cfg *cfg, const snake_state *st, int64_t num_envs, void *stream);

/* Releases what the library keeps for this state (the background spawn-ahead
 * stream and events, created by its first snake_step): waits for its last
 * spawn kernel on the host, then destroys them. Call before freeing the state
 * buffers; a later snake_step on the same buffers creates them afresh. */
int snake_release(const snake_cfg *cfg, const snake_state *st, int64_t num_envs);

/* RGB image of every env's current grid: rgb_from_grid(grid, Cell, CellColors)
 * (grid_util.py:164-175), the frame of SnakeEnv.render('rgb_array') and of the
 * 'gif' frames via image_from_grid (snake_env.py:284-293). palette is HOST
 * memory, uint8 [6][16][3]: the colour of a cell of code v % 10 owned by snake
 * v / 10, i.e. CellColors[code][id % len] * 0.7 ** (id // len) truncated to
 * uint8 (snake.py:14-30), precomputed by the caller with the reference's own
 * arithmetic. rgb is device uint8 [N][H][W][3]. */
int snake_render_rgb(const snake_cfg *cfg, const snake_state *st, int64_t num_envs,
                     const uint8_t *palette, uint8_t *rgb, void *stream);

/* Profiling aid. While enabled, every kernel launch of snake_step / snake_reset
 * is bracketed by timing events on its own stream. snake_timing_read returns the
 * summed device time (ms) and the launch count of one kernel ("k_logic",
 * "k_post", "k_autoreset", "k_encode", "k_spawn", "k_reset") since its last read, and the number of
 * auto-resets run (kernel "resets": count only, every step); it waits for the
 * events. "resets_timed", "spawn_hits" and "spawn_jobs" count, while enabled,
 * the auto-resets, those that started from a ready spawn-ahead record and the
 * spawn-ahead attempts run; "spawn_void", "reset_partial", "respawn_slow",
 * "respawn_slow2", "gate_shut", "draw_wait" (resets that found a background job
 * drawing their record and waited) and "draw_timeout" (... and gave up waiting,
 * drawing from the env's own MT state) are further diagnostic counts. */
int snake_timing_enable(int on);
int snake_timing_read(const char *kernel, double *total_ms, int64_t *count);

/* Testing aid (no reference counterpart), process-wide, read at each
 * snake_step: "draw_wait_ticks" = how long (100 MHz ticks, default 200000 =
 * 2 ms) an auto-reset waits for a background spawn-ahead job drawing its record
 * before it voids the job and draws itself (0: never waits); "spawn_delay_ticks"
 * = fault injection: each background job sleeps that long (default 0) once it
 * has marked a record DRAWING, so resets meet jobs in flight; "fused" = 1 runs
 * the step as one launch (k_step) where the configuration allows it (one
 * frame, at most 4 snakes, table encode, in-step spawn-ahead; default 0);
 * "fuse_roles" = which of k_step's roles run (diagnostics; 7 = all). Results
 * are the same for any values of the first three. Returns SNAKE_E_ARG for an unknown name or a value out of
 * range. */
int snake_debug_set(const char *name, long long value);

/* ---- Fused consumer: the reference's DQN forward on the observation batch
 * (train_dqn.py:104-151 DQN.forward / forward_features, train_ga.py:60-100),
 * conv1 c->32, conv2 32->64, conv3 64->64 (3x3, pad 1, ReLU), NCHW flatten,
 * fc1 64hw->256, fc2 256->128 (ReLU), fc3 128->A, on the bf16 matrix cores with
 * fp32 accumulation (weights and activations rounded to bf16 between layers).
 * obs: uint8 [B][h][w][c] (the env's NHWC per-snake observations, 0/1 values:
 * the reference's /255 branch is not taken). h = w = 2*vision_range+1 with
 * vision_range in [1, 5], c = 8*frame_stack <= 32, A <= 4. */
typedef struct {
    int32_t height, width, channels, num_actions;
    int32_t conv_waves;     /* waves per observation in the conv kernel: 1, 2, 4; 0 = default (4,
                             * or 2 when the row-tile count is odd; SNAKE_DQN_WAVES overrides 0) */
} snake_dqn_cfg;

typedef struct {        /* sizes for snake_dqn_forward (element counts) */
    int64_t conv1_w;    /* bf16 B[32][k1]: k = tap*cpad + channel, tap = ky*3 + kx, zero padded */
    int64_t conv2_w;    /* bf16 B[64][288]: k = tap*32 + channel */
    int64_t conv3_w;    /* bf16 B[64][576]: k = tap*64 + channel; all three stored in MFMA
                         * fragment order: element (o, k) at
                         * ((o/16 * K/32 + k/32) * 4 + (k%32)/8) * 128 + (o%16) * 8 + k%8 */
    int64_t fc1_w;      /* bf16 [256][64*p16], k in conv3's MFMA fragment order:
                         * k = m*1024 + half*512 + quad*128 + c16*8 + j*4 + r holds
                         * channel (2*half + j)*16 + c16 at GEMM row i = m*16 + 4*quad + r,
                         * i.e. at observation position snake_dqn_rows()[i] (zero weights
                         * where that is -1) */
    int64_t fc2_w;      /* bf16 [128][256] */
    int64_t act_per_obs;/* bf16 scratch per observation: 64*p16 */
    int32_t cpad, p16, k1;   /* channels padded to a power of two >= 8; GEMM rows (16 per tile); 9*cpad to 32 */
    int32_t lds_conv;   /* LDS bytes per conv workgroup */
} snake_dqn_layout;

typedef struct {        /* device weights (layouts in snake_dqn_layout; biases and fc3 fp32) */
    const uint16_t *conv1_w, *conv2_w, *conv3_w, *fc1_w, *fc2_w;
    const float *conv1_b, *conv2_b, *conv3_b, *fc1_b, *fc2_b;
    const float *fc3_w;  /* [A][128] */
    const float *fc3_b;  /* [A] */
} snake_dqn_net;

int snake_dqn_plan(const snake_dqn_cfg *cfg, snake_dqn_layout *out);

/* The convolutions' GEMM row -> observation position map (p = y*w + x, -1 for a
 * padding row): rows[i] for i < p16. Rows are assigned so that the 16 rows of a
 * tile sit in distinct LDS banks (dqn_kernels.hip). Returns p16 (rows may be
 * NULL to query it), < 0 on error. */
int64_t snake_dqn_rows(const snake_dqn_cfg *cfg, int32_t *rows, int64_t n);

/* q_out: float [B][A]; feat_out (may be NULL): float [B][128] = forward_features;
 * act_scratch: bf16 [B][act_per_obs] device buffer. Two launches on `stream`. */
int snake_dqn_forward(const snake_dqn_cfg *cfg, const snake_dqn_net *net, const uint8_t *obs,
                      int64_t batch, uint16_t *act_scratch, float *q_out, float *feat_out,
                      void *stream);

/* fp32 mode of the DQN consumer (dqn32_kernels.hip): the same network in fp32
 * arithmetic (fp32 matrix cores: exact fp32 products, fp32 sums) on any observation size (e.g. train_dqn.py's 20x20 full map,
 * :29-33), cfg->channels a multiple of 8, conv_waves ignored. Weights fp32,
 * row-major [out][in]: conv w [cout][9*cin] with k = (ky*3 + kx)*cin + ci;
 * fc1 [256][h*w*64] with column p*64 + ch (the reference's NCHW flatten
 * column ch*h*w + p, permuted once); fc2 [128][256]; fc3 [A][128]. The uint8
 * input is divided by 255 when the batch holds a value > 1 (train_dqn.py:122). */
typedef struct {
    const float *conv1_w, *conv2_w, *conv3_w, *fc1_w, *fc2_w, *fc3_w;
    const float *conv1_b, *conv2_b, *conv3_b, *fc1_b, *fc2_b, *fc3_b;
} snake_dqn32_net;

/* Device scratch bytes snake_dqn32_forward needs for `batch` observations (< 0 on error). */
int64_t snake_dqn32_scratch(const snake_dqn_cfg *cfg, int64_t batch);

/* q_out: float [B][A]; feat_out (may be NULL): float [B][128]. Seven launches on `stream`. */
int snake_dqn32_forward(const snake_dqn_cfg *cfg, const snake_dqn32_net *net, const uint8_t *obs,
                        int64_t batch, void *scratch, float *q_out, float *feat_out, void *stream);

/* Last error message of this thread ("" if none). */
const char *snake_last_error(void);

int snake_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* SNAKE_ENV_H */
