/*
 * snake_oracle.c -- serial CPU restatement of the reference SnakeEnv.
 *
 * TEST INFRASTRUCTURE ONLY (see snake_oracle.h): the parity checker and the
 * bench.py cpu_baseline ("port"). Never linked into the product.
 *
 * Every function cites the reference line it restates
 * (paths relative to /root/reference/marlenv/marlenv/).
 * Build: make -C oracle   (gcc -O2 -ffp-contract=off; float64 order of ops kept).
 */
#include "snake_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ MT19937
 * numpy legacy RandomState bit generator (numpy/random/src/mt19937/mt19937.c,
 * numpy/random/src/legacy + distributions.c), pinned numpy==1.21.0
 * (requirements.txt:2). The stream is frozen by numpy's compatibility policy.
 */
#define MT_N 624
#define MT_M 397
typedef struct { uint32_t key[MT_N]; int pos; } so_mt;

static void mt_seed(so_mt *st, uint32_t seed)            /* mt19937_seed == init_genrand */
{
    for (int pos = 0; pos < MT_N; pos++) {
        st->key[pos] = seed;
        seed = 1812433253U * (seed ^ (seed >> 30)) + (uint32_t)pos + 1U;
    }
    st->pos = MT_N;
}

static void mt_twist(so_mt *st)                          /* mt19937_gen */
{
    uint32_t *k = st->key, y;
    int i;
    for (i = 0; i < MT_N - MT_M; i++) {
        y = (k[i] & 0x80000000U) | (k[i + 1] & 0x7fffffffU);
        k[i] = k[i + MT_M] ^ (y >> 1) ^ (-(y & 1U) & 0x9908b0dfU);
    }
    for (; i < MT_N - 1; i++) {
        y = (k[i] & 0x80000000U) | (k[i + 1] & 0x7fffffffU);
        k[i] = k[i + (MT_M - MT_N)] ^ (y >> 1) ^ (-(y & 1U) & 0x9908b0dfU);
    }
    y = (k[MT_N - 1] & 0x80000000U) | (k[0] & 0x7fffffffU);
    k[MT_N - 1] = k[MT_M - 1] ^ (y >> 1) ^ (-(y & 1U) & 0x9908b0dfU);
    st->pos = 0;
}

static uint32_t mt_next(so_mt *st)                       /* mt19937_next (tempering) */
{
    if (st->pos == MT_N) mt_twist(st);
    uint32_t y = st->key[st->pos++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680U;
    y ^= (y << 15) & 0xefc60000U;
    y ^= (y >> 18);
    return y;
}

static uint32_t gen_mask(uint32_t max)                   /* smallest 2^k-1 >= max */
{
    uint32_t m = max;
    m |= m >> 1; m |= m >> 2; m |= m >> 4; m |= m >> 8; m |= m >> 16;
    return m;
}

/* random_interval(max): used by RandomState.shuffle -> permutation (snake_env.py:581) */
static uint32_t mt_interval(so_mt *st, uint32_t max)
{
    if (max == 0) return 0;
    uint32_t mask = gen_mask(max), v;
    while ((v = (mt_next(st) & mask)) > max) {}
    return v;
}

/* randint(0, n, size=k), legacy int64 masked path (grid_util.py:130):
 * rng = n-1; rng == 0 -> zeros and NO draw; rng == 0xffffffff -> raw draw;
 * else masked rejection per value. n <= 2^32 here (grid cells). */
static void mt_randint(so_mt *st, int64_t n, int64_t k, int64_t *out)
{
    uint64_t rng = (uint64_t)(n - 1);
    if (rng == 0) { for (int64_t i = 0; i < k; i++) out[i] = 0; return; }
    if (rng == 0xffffffffULL) { for (int64_t i = 0; i < k; i++) out[i] = mt_next(st); return; }
    uint32_t mask = gen_mask((uint32_t)rng), v;
    for (int64_t i = 0; i < k; i++) {
        while ((v = (mt_next(st) & mask)) > (uint32_t)rng) {}
        out[i] = v;
    }
}

/* permutation(n) = shuffle(arange(n)): for i = n-1 .. 1: j = random_interval(i); swap */
static void mt_permutation(so_mt *st, int64_t n, int64_t *arr)
{
    for (int64_t i = 0; i < n; i++) arr[i] = i;
    for (int64_t i = n - 1; i >= 1; i--) {
        int64_t j = mt_interval(st, (uint32_t)i);
        int64_t t = arr[j]; arr[j] = arr[i]; arr[i] = t;
    }
}

/* --------------------------------------------------------------- constants
 * Cell (core/snake.py:5-11); Direction (core/snake.py:33-37) as (dr, dc).
 */
enum { EMPTY = 0, WALL = 1, FRUIT = 2, HEAD = 3, BODY = 4, TAIL = 5 };
static const int DR[4] = {-1, 0, 1, 0};   /* UP, RIGHT, DOWN, LEFT */
static const int DC[4] = {0, 1, 0, -1};

static int dir_of(int dr, int dc)
{
    for (int d = 0; d < 4; d++) if (DR[d] == dr && DC[d] == dc) return d;
    return -1;   /* Direction(...) would raise ValueError */
}

/* -------------------------------------------------------- DFS candidates
 * grid_util.py:7-11 SHIFTS = [(0,1),(1,0),(0,-1),(-1,0)] (named DOWN/RIGHT/UP/LEFT there);
 * dfs_sweep_empty :73-80, _dfs_helper :83-99, _head_blocked :102-110, _inbound :113-115.
 */
static const int SH_R[4] = {0, 1, 0, -1};
static const int SH_C[4] = {1, 0, -1, 0};

typedef struct {
    int H, W, L;
    const uint8_t *empty;   /* make_grid(...) == 0 */
    int16_t *out;           /* may be NULL (count only) */
    int64_t count;
    int hist_r[64], hist_c[64];
} dfs_ctx;

static int in_hist(const dfs_ctx *c, int n, int r, int cc)
{
    for (int i = 0; i < n; i++) if (c->hist_r[i] == r && c->hist_c[i] == cc) return 1;
    return 0;
}

static int inbound(const dfs_ctx *c, int r, int cc)
{
    return r >= 0 && cc >= 0 && r < c->H && cc < c->W;
}

static int head_blocked(const dfs_ctx *c, int n, int xr, int xc)   /* :102-110 */
{
    int blocked = 0;
    for (int s = 0; s < 4; s++) {
        int r = c->hist_r[0] + SH_R[s], cc = c->hist_c[0] + SH_C[s];
        /* the reference reads mask[node] before the inbound test; first_node is
         * interior (walls are never empty) so node is always in range */
        if (!inbound(c, r, cc) || c->empty[r * c->W + cc] == 0 || in_hist(c, n, r, cc) ||
            (r == xr && cc == xc))
            blocked++;
    }
    return blocked == 4;
}

static void dfs_helper(dfs_ctx *c, int n, int r, int cc)           /* :83-99 */
{
    c->hist_r[n] = r; c->hist_c[n] = cc; n++;
    if (n == c->L) {
        if (c->out) {
            for (int i = 0; i < n; i++) {
                c->out[(c->count * c->L + i) * 2 + 0] = (int16_t)c->hist_r[i];
                c->out[(c->count * c->L + i) * 2 + 1] = (int16_t)c->hist_c[i];
            }
        }
        c->count++;
        return;
    }
    for (int s = 0; s < 4; s++) {
        int rr = r + SH_R[s], ccc = cc + SH_C[s];
        if (inbound(c, rr, ccc) && !in_hist(c, n, rr, ccc) && c->empty[rr * c->W + ccc]) {
            if (!head_blocked(c, n, rr, ccc)) dfs_helper(c, n, rr, ccc);   /* deepcopy(history) */
        }
    }
}

int64_t so_candidates(int32_t H, int32_t W, int32_t L, int16_t *out)  /* dfs_sweep_empty */
{
    if (L < 1 || L > 64) return -1;
    uint8_t *empty = (uint8_t *)calloc((size_t)H * W, 1);
    for (int r = 1; r < H - 1; r++)
        for (int c = 1; c < W - 1; c++) empty[r * W + c] = 1;   /* make_grid :14-20 */
    dfs_ctx c = {H, W, L, empty, out, 0, {0}, {0}};
    for (int r = 0; r < H; r++)
        for (int cc = 0; cc < W; cc++)
            if (empty[r * W + cc]) dfs_helper(&c, 0, r, cc);
    free(empty);
    return c.count;
}

/* -------------------------------------------------------------------- Snake
 * core/snake.py:52-107. Body = head coord + deque of directions; directions[0]
 * points from coords[1] to the head. Kept as a ring of direction indices.
 */
typedef struct {
    int hr, hc, tr, tc, dir;
    int alive, fruit, death, kills, win;
    int *dq; int dq_head, dq_len, dq_cap;
} so_snake;

static void dq_appendleft(so_snake *s, int d)
{
    s->dq_head = (s->dq_head + s->dq_cap - 1) % s->dq_cap;
    s->dq[s->dq_head] = d;
    s->dq_len++;
}

static int dq_pop(so_snake *s)
{
    int d = s->dq[(s->dq_head + s->dq_len - 1) % s->dq_cap];
    s->dq_len--;
    return d;
}

static int dq_at(const so_snake *s, int i) { return s->dq[(s->dq_head + i) % s->dq_cap]; }

static void snake_reset_reward_state(so_snake *s)        /* snake.py:79-84 */
{
    s->fruit = 0; s->death = 0; s->kills = 0; s->win = 0;
}

static void snake_init(so_snake *s, const int *cr, const int *cc, int n)   /* snake.py:53-74 */
{
    s->hr = cr[0]; s->hc = cc[0];
    s->tr = cr[n - 1]; s->tc = cc[n - 1];
    s->dir = dir_of(cr[0] - cr[1], cc[0] - cc[1]);
    s->dq_head = 0; s->dq_len = 0;
    for (int i = 1; i < n; i++) s->dq[s->dq_len++] = dir_of(cr[i - 1] - cr[i], cc[i - 1] - cc[i]);
    s->alive = 1;
    snake_reset_reward_state(s);
}

/* coords property, snake.py:86-94; returns count */
static int snake_coords(const so_snake *s, int *rr, int *cc)
{
    int r = s->hr, c = s->hc, n = 0;
    rr[n] = r; cc[n] = c; n++;
    for (int i = 0; i < s->dq_len; i++) {
        int d = dq_at(s, i);
        r -= DR[d]; c -= DC[d];
        rr[n] = r; cc[n] = c; n++;
    }
    return n;
}

/* move(), snake.py:96-107; returns 1 and the previous tail when the tail moved */
static int snake_move(so_snake *s, int *ptr, int *ptc)
{
    s->hr += DR[s->dir]; s->hc += DC[s->dir];
    dq_appendleft(s, s->dir);
    int moved = 0;
    if (!s->fruit) {
        *ptr = s->tr; *ptc = s->tc; moved = 1;
        int td = dq_pop(s);
        s->tr += DR[td]; s->tc += DC[td];
    }
    snake_reset_reward_state(s);
    return moved;
}

/* ---------------------------------------------------------------------- env */
struct so_env {
    so_cfg cfg;
    int H, W, S, oh, ow, fs;
    so_mt mt;
    int *grid;                       /* int64 in the reference; values <= 10*(S-1)+5 */
    so_snake *snakes;
    int64_t alive_snakes, episode_length;
    double *epi_scores, *epi_steps, *epi_fruits, *epi_kills;
    int64_t n_cand; int16_t *cand;   /* dfs_sweep_empty(make_grid(H,W), L) */
    uint8_t *frames;                 /* self.obs deque(maxlen=fs): fs x S x oh x ow x 8 */
    int64_t frame_sz;                /* S*oh*ow*8 */
    int next_dir[4][3];              /* _next_direction table, from the reference's trig */
    /* scratch */
    int *cr, *cc, *perm_buf_i;
    int64_t *perm;
    int64_t *ibuf;
    float *full;                     /* one snake's H x W x 8 _encode plane */
};

/* _next_direction, snake_env.py:598-608: angle = atan2(dc, dr) (note the (value[1],
 * value[0]) argument order), new = (int(cos(angle+a)), int(sin(angle+a))) with the
 * action_angle_dict :40-44 {0: 0, 1: pi/2, 2: -pi/2}; int() truncates toward zero. */
static void build_next_dir(so_env *e)
{
    const double ang[3] = {0.0, M_PI / 2.0, -M_PI / 2.0};
    for (int d = 0; d < 4; d++) {
        double angle = atan2((double)DC[d], (double)DR[d]);
        for (int a = 0; a < 3; a++) {
            int nr = (int)cos(angle + ang[a]);
            int nc = (int)sin(angle + ang[a]);
            e->next_dir[d][a] = dir_of(nr, nc);
        }
    }
}

/* _next_direction_global, snake_env.py:610-632 ('human' observer) */
static int next_dir_global(int d, int action)
{
    int nd = d;
    if (DR[d] == 0) {            /* direction.value[0] == 0 */
        if (action == 3) nd = 2;           /* DOWN */
        else if (action == 4) nd = 0;      /* UP */
    } else if (DC[d] == 0) {     /* direction.value[1] == 0 */
        if (action == 1) nd = 3;           /* LEFT */
        else if (action == 2) nd = 1;      /* RIGHT */
    }
    return nd;
}

so_env *so_create(const so_cfg *cfg, uint32_t seed)
{
    if (cfg->num_snakes < 1 || cfg->num_snakes > 16 || cfg->snake_length < 2 ||
        cfg->frame_stack < 1 || cfg->num_fruits < 1 || cfg->height < 3 || cfg->width < 3)
        return NULL;
    so_env *e = (so_env *)calloc(1, sizeof(so_env));
    e->cfg = *cfg;
    e->H = cfg->height; e->W = cfg->width; e->S = cfg->num_snakes; e->fs = cfg->frame_stack;
    if (cfg->vision_range > 0) { e->oh = e->ow = 2 * cfg->vision_range + 1; }   /* :115-129 */
    else { e->oh = e->H; e->ow = e->W; }
    mt_seed(&e->mt, seed);                                    /* np.random.seed(seed) */
    int HW = e->H * e->W;
    e->grid = (int *)calloc(HW, sizeof(int));
    e->snakes = (so_snake *)calloc(e->S, sizeof(so_snake));
    for (int k = 0; k < e->S; k++) {
        e->snakes[k].dq_cap = HW + 1;
        e->snakes[k].dq = (int *)calloc(HW + 1, sizeof(int));
    }
    e->epi_scores = (double *)calloc(e->S, sizeof(double));
    e->epi_steps = (double *)calloc(e->S, sizeof(double));
    e->epi_fruits = (double *)calloc(e->S, sizeof(double));
    e->epi_kills = (double *)calloc(e->S, sizeof(double));
    e->n_cand = so_candidates(e->H, e->W, cfg->snake_length, NULL);
    e->cand = (int16_t *)malloc(sizeof(int16_t) * 2 * cfg->snake_length * (e->n_cand + 1));
    so_candidates(e->H, e->W, cfg->snake_length, e->cand);
    e->frame_sz = (int64_t)e->S * e->oh * e->ow * 8;
    e->frames = (uint8_t *)calloc((size_t)e->frame_sz * e->fs, 1);
    e->cr = (int *)calloc(HW + 1, sizeof(int));
    e->cc = (int *)calloc(HW + 1, sizeof(int));
    e->perm = (int64_t *)calloc(e->n_cand + 1, sizeof(int64_t));
    e->ibuf = (int64_t *)calloc(HW + 64, sizeof(int64_t));
    e->full = (float *)calloc((size_t)HW * 8, sizeof(float));
    build_next_dir(e);
    e->episode_length = 0;
    return e;
}

void so_destroy(so_env *e)
{
    if (!e) return;
    for (int k = 0; k < e->S; k++) free(e->snakes[k].dq);
    free(e->grid); free(e->snakes); free(e->epi_scores); free(e->epi_steps);
    free(e->epi_fruits); free(e->epi_kills); free(e->cand); free(e->frames);
    free(e->cr); free(e->cc); free(e->perm); free(e->ibuf); free(e->full);
    free(e);
}

int64_t so_obs_size(const so_env *e) { return e->frame_sz * e->fs; }

/* _encode, snake_env.py:474-519: per snake 8 channels
 * [wall, fruit, other head, other body, other tail, own head, own body, own tail],
 * then the zero-padded (2vr+1)^2 crop centred on argmax(own head channel). */
static void encode_frame(so_env *e, uint8_t *dst /* S x oh x ow x 8 */)
{
    const int H = e->H, W = e->W, S = e->S;
    const int vr = e->cfg.vision_range;
    for (int k = 0; k < S; k++) {
        float *full = e->full;
        memset(full, 0, sizeof(float) * H * W * 8);
        for (int r = 0; r < H; r++) {
            for (int c = 0; c < W; c++) {
                int v = e->grid[r * W + c];
                float *px = full + (r * W + c) * 8;
                if (v == WALL || v == FRUIT) {
                    px[v - 1] = 1.0f;                       /* env_objs[r,c,v-1] = 1 */
                } else if (v != EMPTY) {
                    int sid = v / 10, obj = v % 10;
                    float myself = (sid == k) ? 1.0f : 0.0f;
                    px[2 + obj] = myself;                   /* snake_objs[.., obj_id, :] */
                    px[2 + obj - 3] = 1.0f - myself;        /* snake_objs[.., obj_id-3, :] */
                }
            }
        }
        uint8_t *o = dst + (int64_t)k * e->oh * e->ow * 8;
        if (!vr) {
            for (int i = 0; i < H * W * 8; i++) o[i] = (uint8_t)full[i];
            continue;
        }
        /* head_pos = unravel(argmax(full[:,:,5])): first maximum, (0,0) if all zero */
        int best = 0;
        for (int i = 0; i < H * W; i++)
            if (full[i * 8 + 5] > full[best * 8 + 5]) best = i;
        int hr = best / W, hc = best % W;
        int minr = hr - vr < 0 ? 0 : hr - vr, minc = hc - vr < 0 ? 0 : hc - vr;
        int maxr = hr + vr > H - 1 ? H - 1 : hr + vr, maxc = hc + vr > W - 1 ? W - 1 : hc + vr;
        int sr = minr - hr + vr, sc = minc - hc + vr;
        int D = 2 * vr + 1;
        memset(o, 0, (size_t)D * D * 8);
        for (int r = minr; r <= maxr; r++)
            for (int c = minc; c <= maxc; c++)
                for (int ch = 0; ch < 8; ch++)
                    o[((sr + r - minr) * D + (sc + c - minc)) * 8 + ch] =
                        (uint8_t)full[(r * W + c) * 8 + ch];
    }
}

/* _get_obs / _init_obs (:444-472): deque(maxlen=fs) of frames; output per snake is
 * the channel concat of the frames, oldest first; then np.array(obs, uint8) (:414). */
static void emit_obs(so_env *e, uint8_t *obs)
{
    const int S = e->S, P = e->oh * e->ow, fs = e->fs;
    for (int k = 0; k < S; k++)
        for (int p = 0; p < P; p++)
            for (int f = 0; f < fs; f++)
                memcpy(obs + (((int64_t)k * P + p) * fs + f) * 8,
                       e->frames + (int64_t)f * e->frame_sz + ((int64_t)k * P + p) * 8, 8);
}

static void init_obs(so_env *e, uint8_t *obs)           /* :444-459 */
{
    encode_frame(e, e->frames);
    for (int f = 1; f < e->fs; f++) memcpy(e->frames + f * e->frame_sz, e->frames, e->frame_sz);
    if (obs) emit_obs(e, obs);
}

static void get_obs(so_env *e, uint8_t *obs)            /* :461-472 */
{
    if (e->fs > 1) memmove(e->frames, e->frames + e->frame_sz, (size_t)e->frame_sz * (e->fs - 1));
    encode_frame(e, e->frames + (int64_t)(e->fs - 1) * e->frame_sz);
    if (obs) emit_obs(e, obs);
}

static void reset_epi_stats(so_env *e)                  /* :438-442 */
{
    for (int k = 0; k < e->S; k++)
        e->epi_scores[k] = e->epi_steps[k] = e->epi_fruits[k] = e->epi_kills[k] = 0.0;
}

/* random_empty_coords (grid_util.py:126-133) + grid[xs, ys] = FRUIT.
 * Returns 0 when no empty cell (the reference returns (None, None), no draw). */
static int place_fruits(so_env *e, int64_t k)
{
    const int HW = e->H * e->W;
    int64_t n = 0;
    for (int i = 0; i < HW; i++) if (e->grid[i] == EMPTY) e->ibuf[n++] = i;   /* np.where, row-major */
    if (n == 0) return 0;
    int64_t *idx = (int64_t *)malloc(sizeof(int64_t) * (k > 0 ? k : 1));
    mt_randint(&e->mt, n, k, idx);
    for (int64_t i = 0; i < k; i++) e->grid[e->ibuf[idx[i]]] = FRUIT;
    free(idx);
    return 1;
}

/* _generate_snakes, snake_env.py:576-589 (+ _clear_overlap :568-574) */
static void generate_snakes(so_env *e)
{
    const int S = e->S, L = e->cfg.snake_length, HW = e->H * e->W;
    uint8_t *seen = (uint8_t *)calloc(HW, 1);
    for (;;) {
        mt_permutation(&e->mt, e->n_cand, e->perm);
        memset(seen, 0, HW);
        int ok = 1;
        for (int k = 0; k < S && k < e->n_cand; k++) {
            const int16_t *cd = e->cand + e->perm[k] * L * 2;
            for (int i = 0; i < L; i++) {
                int cell = cd[2 * i] * e->W + cd[2 * i + 1];
                if (seen[cell]) ok = 0;
                seen[cell] = 1;
            }
        }
        if (ok) break;
    }
    free(seen);
    for (int k = 0; k < S; k++) {
        const int16_t *cd = e->cand + e->perm[k] * L * 2;
        for (int i = 0; i < L; i++) { e->cr[i] = cd[2 * i]; e->cc[i] = cd[2 * i + 1]; }
        snake_init(&e->snakes[k], e->cr, e->cc, L);
    }
}

int so_reset(so_env *e, uint8_t *obs)                   /* snake_env.py:131-159 */
{
    const int H = e->H, W = e->W;
    for (int r = 0; r < H; r++)                         /* make_grid, grid_util.py:14-20 */
        for (int c = 0; c < W; c++)
            e->grid[r * W + c] = (r == 0 || c == 0 || r == H - 1 || c == W - 1) ? WALL : EMPTY;
    generate_snakes(e);
    for (int k = 0; k < e->S; k++) {                    /* :138-144 */
        so_snake *s = &e->snakes[k];
        int n = snake_coords(s, e->cr, e->cc);
        for (int i = 0; i < n; i++) e->grid[e->cr[i] * W + e->cc[i]] = BODY + 10 * k;
        e->grid[s->hr * W + s->hc] = HEAD + 10 * k;
        e->grid[s->tr * W + s->tc] = TAIL + 10 * k;
    }
    place_fruits(e, e->cfg.num_fruits);                 /* :147-148 */
    e->alive_snakes = e->S;
    init_obs(e, obs);
    reset_epi_stats(e);
    e->episode_length = 0;
    return 0;
}

/* draw(grid, coords, value), grid_util.py:148-161 */
static int draw_cells(so_env *e, const int *rr, const int *cc, int n, int value)
{
    for (int i = 0; i < n; i++)
        if (rr[i] == 0 || rr[i] == e->H - 1 || cc[i] == 0 || cc[i] == e->W - 1) return 0;
    for (int i = 0; i < n; i++) e->grid[rr[i] * e->W + cc[i]] = value;
    return 1;
}

/* _update_grid, snake_env.py:546-566 */
static void update_grid(so_env *e, int k)
{
    so_snake *s = &e->snakes[k];
    const int W = e->W, id = 10 * k;
    if (s->alive) {
        e->grid[s->hr * W + s->hc] = BODY + id;
        int ptr, ptc;
        if (snake_move(s, &ptr, &ptc)) {
            if (e->grid[ptr * W + ptc] == TAIL + id) e->grid[ptr * W + ptc] = EMPTY;
        }
        e->grid[s->hr * W + s->hc] = HEAD + id;
        e->grid[s->tr * W + s->tc] = TAIL + id;
    } else {
        int n = snake_coords(s, e->cr, e->cc);
        if (e->grid[e->cr[n - 1] * W + e->cc[n - 1]] / 10 != k) n--;
        draw_cells(e, e->cr, e->cc, n, EMPTY);     /* 'draw failed' print on False */
        int ptr, ptc;
        snake_move(s, &ptr, &ptc);
    }
}

int so_step(so_env *e, const int32_t *actions, uint8_t *obs, double *rews, uint8_t *dones,
            so_info *info)
{
    const int S = e->S, W = e->W;
    /* next_head_coords: dict coord -> [idx], insertion-ordered (:318-330) */
    int g_cell[16], g_n = 0, g_cnt[16], g_idx[16][16];
    for (int k = 0; k < S; k++) {
        so_snake *s = &e->snakes[k];
        if (!s->alive) continue;
        int a = actions[k];
        if (e->cfg.observer == 1) {
            s->dir = next_dir_global(s->dir, a);
        } else {
            if (a < 0 || a > 2) return -1;                /* action_angle_dict[action] KeyError */
            s->dir = e->next_dir[s->dir][a];
        }
        int cell = (s->hr + DR[s->dir]) * W + (s->hc + DC[s->dir]);
        int g;
        for (g = 0; g < g_n; g++) if (g_cell[g] == cell) break;
        if (g == g_n) { g_cell[g_n] = cell; g_cnt[g_n] = 0; g_n++; }
        g_idx[g][g_cnt[g]++] = k;
    }
    /* _check_collision :521-544 */
    int dead[16], n_dead = 0, fruit_idx[16], n_fruit = 0;
    int64_t fruit_taken = 0;
    for (int g = 0; g < g_n; g++) {
        int v = e->grid[g_cell[g]];
        int cv = v % 10;
        if (g_cnt[g] > 1 || cv == WALL || cv == BODY || cv == HEAD) {
            for (int i = 0; i < g_cnt[g]; i++) dead[n_dead++] = g_idx[g][i];
            if (cv == FRUIT) fruit_taken++;
            if (cv == BODY || cv == HEAD) e->snakes[v / 10].kills++;
        } else if (g_cnt[g] == 1 && cv == FRUIT) {
            fruit_idx[n_fruit++] = g_idx[g][0];
            fruit_taken++;
        }
    }
    /* :334-352 */
    e->alive_snakes -= n_dead;     /* list(set(dead)): idxs are already unique */
    for (int i = 0; i < n_dead; i++) { e->snakes[dead[i]].death = 1; e->snakes[dead[i]].alive = 0; }
    for (int i = 0; i < n_fruit; i++) {
        so_snake *s = &e->snakes[fruit_idx[i]];
        int tcell = s->tr * W + s->tc;
        for (int g = 0; g < g_n; g++) {
            if (g_cell[g] != tcell) continue;
            for (int j = 0; j < g_cnt[g]; j++) {
                so_snake *d = &e->snakes[g_idx[g][j]];
                d->death = 1; d->alive = 0;
                e->alive_snakes -= 1;
                s->kills += 1;
            }
        }
        s->fruit = 1;
    }
    if (e->alive_snakes == 1 && S > 1) {
        for (int k = 0; k < S; k++) if (e->snakes[k].alive) { e->snakes[k].win = 1; break; }
    }
    /* rewards + grid update, in snake index order (:354-374) */
    double fr[16], kl[16];
    uint8_t dn[16];
    const so_cfg *c = &e->cfg;
    for (int k = 0; k < S; k++) {
        so_snake *s = &e->snakes[k];
        if (!s->death && !s->alive) {
            rews[k] = 0.0; fr[k] = 0.0; kl[k] = 0.0;
        } else {
            double r = c->rew_time * (double)s->alive;
            r += c->rew_fruit * (double)s->fruit;
            r += c->rew_lose * (double)s->death;
            r += c->rew_kill * (double)s->kills;
            r += c->rew_win * (double)s->win;
            rews[k] = r;
            fr[k] = (double)s->fruit;
            kl[k] = (double)s->kills;
            update_grid(e, k);
        }
        dn[k] = !s->alive;
    }
    if (fruit_taken) place_fruits(e, fruit_taken);      /* :376-379 */
    get_obs(e, obs);                                    /* :381 */
    for (int k = 0; k < S; k++) {                       /* :385-389 */
        double m = 1.0 - (double)dn[k];
        e->epi_scores[k] = e->epi_scores[k] + m * rews[k];
        e->epi_steps[k] = e->epi_steps[k] + m * 1.0;
        e->epi_fruits[k] = e->epi_fruits[k] + m * fr[k];
        e->epi_kills[k] = e->epi_kills[k] + m * kl[k];
    }
    e->episode_length += 1;                             /* :392-394 */
    if ((double)e->episode_length >= c->max_episode_steps)
        for (int k = 0; k < S; k++) dn[k] = 1;
    /* _done_fn (:416-417): all(dones); CoopSnakeEnv._done_fn any(dones), and its
     * step() then reports every done True (coop_snake_env.py:14-22) -- after the
     * statistics above were masked with the per-snake dones */
    int all = 1, any = 0;
    for (int k = 0; k < S; k++) { all &= dn[k]; any |= dn[k]; }
    const int ended = c->coop ? any : all;
    for (int k = 0; k < S; k++) dones[k] = (c->coop && ended) ? 1 : dn[k];
    if (!ended) return 0;
    /* :396-412 competition rank on descending unique scores */
    if (info) {
        int assigned[16] = {0};
        int64_t base = 1;
        for (;;) {
            int found = 0; double best = 0;
            for (int k = 0; k < S; k++)
                if (!assigned[k] && (!found || e->epi_scores[k] > best)) { best = e->epi_scores[k]; found = 1; }
            if (!found) break;
            int64_t cnt = 0;
            for (int k = 0; k < S; k++)
                if (!assigned[k] && e->epi_scores[k] == best) { info->rank[k] = base; assigned[k] = 1; cnt++; }
            base += cnt;
        }
        for (int k = 0; k < S; k++) {
            info->scores[k] = e->epi_scores[k]; info->steps[k] = e->epi_steps[k];
            info->fruits[k] = e->epi_fruits[k]; info->kills[k] = e->epi_kills[k];
        }
    }
    reset_epi_stats(e);
    return 1;
}

void so_get_grid(const so_env *e, uint8_t *out)
{
    for (int i = 0; i < e->H * e->W; i++) out[i] = (uint8_t)e->grid[i];   /* <= 155 for S <= 16 */
}

int64_t so_alive_snakes(const so_env *e) { return e->alive_snakes; }
int64_t so_episode_length(const so_env *e) { return e->episode_length; }

void so_get_snakes(const so_env *e, int32_t *out)
{
    for (int k = 0; k < e->S; k++) {
        const so_snake *s = &e->snakes[k];
        int32_t *o = out + 7 * k;
        o[0] = s->hr; o[1] = s->hc; o[2] = s->tr; o[3] = s->tc; o[4] = s->dir;
        o[5] = s->alive; o[6] = s->dq_len + 1;
    }
}

int so_inject(so_env *e, const int32_t *grid, const int32_t *coords, const int32_t *off,
              const uint8_t *alive, int64_t alive_snakes, int64_t episode_length)
{
    for (int i = 0; i < e->H * e->W; i++) e->grid[i] = grid[i];
    for (int k = 0; k < e->S; k++) {
        int n = off[k + 1] - off[k];
        if (n < 2) return -1;
        for (int i = 0; i < n; i++) { e->cr[i] = coords[2 * (off[k] + i)]; e->cc[i] = coords[2 * (off[k] + i) + 1]; }
        snake_init(&e->snakes[k], e->cr, e->cc, n);
        e->snakes[k].alive = alive[k];
    }
    e->alive_snakes = alive_snakes;
    init_obs(e, NULL);
    reset_epi_stats(e);
    e->episode_length = episode_length;
    return 0;
}

void so_rng_raw(uint32_t seed, int64_t n, uint32_t *out)
{
    so_mt st; mt_seed(&st, seed);
    for (int64_t i = 0; i < n; i++) out[i] = mt_next(&st);
}

void so_rng_randint(uint32_t seed, int64_t n, int64_t k, int64_t *out, uint32_t *next)
{
    so_mt st; mt_seed(&st, seed);
    mt_randint(&st, n, k, out);
    *next = mt_next(&st);
}

void so_rng_permutation(uint32_t seed, int64_t n, int64_t *out, uint32_t *next)
{
    so_mt st; mt_seed(&st, seed);
    mt_permutation(&st, n, out);
    *next = mt_next(&st);
}

/* CPU baseline driver (bench.py cpu_baseline, scripts/cpu_ratio.py): n_env envs
 * seeded seed..seed+n_env-1, stepped round-robin for `steps` steps each with
 * uniform random actions in {0,1,2} (xorshift32, act_seed), reset whenever all
 * dones are True (the vector-env auto-reset, wrappers.py:141-143). Returns the
 * env-steps run, or -1. */
int64_t so_rollout(const so_cfg *cfg, int32_t n_env, uint32_t seed, int64_t steps, uint32_t act_seed)
{
    if (n_env < 1 || n_env > 4096) return -1;
    so_env **envs = (so_env **)calloc((size_t)n_env, sizeof *envs);
    if (!envs) return -1;
    int64_t n = -1;
    uint8_t *obs = NULL;
    for (int i = 0; i < n_env; i++)
        if (!(envs[i] = so_create(cfg, seed + (uint32_t)i))) goto done;
    obs = (uint8_t *)malloc((size_t)so_obs_size(envs[0]));
    if (!obs) goto done;
    for (int i = 0; i < n_env; i++) so_reset(envs[i], obs);
    uint32_t x = act_seed ? act_seed : 12345u;
    int32_t act[16];
    double rews[16];
    uint8_t dones[16];
    n = 0;
    for (int64_t t = 0; t < steps; t++) {
        for (int i = 0; i < n_env; i++) {
            for (int k = 0; k < cfg->num_snakes; k++) {
                x ^= x << 13; x ^= x >> 17; x ^= x << 5;
                act[k] = (int32_t)(x % 3u);
            }
            int rc = so_step(envs[i], act, obs, rews, dones, NULL);
            int all = 1;
            for (int k = 0; k < cfg->num_snakes; k++) all &= dones[k];
            if (rc >= 0 && all) so_reset(envs[i], obs);
            n++;
        }
    }
done:
    for (int i = 0; i < n_env; i++) if (envs[i]) so_destroy(envs[i]);
    free(envs);
    free(obs);
    return n;
}

/* ---- batch checker (tests/test_gpu_parity.py full-size cases) ------------
 * n envs seeded seed+i, every env stepped with its own actions and reset when
 * its episode ends (all dones; any under coop), the vector-env auto-reset
 * (wrappers.py:141-143): the reset obs replaces the step's, rewards/dones and the
 * episode summary stay the step's. Envs are split over nthreads pthreads. */
#include <pthread.h>

struct so_batch {
    so_cfg cfg;
    int64_t n, obs_sz;
    so_env **envs;
};

so_batch *so_batch_create(const so_cfg *cfg, int64_t n, uint32_t seed)
{
    if (n < 1) return NULL;
    so_batch *b = (so_batch *)calloc(1, sizeof *b);
    if (!b) return NULL;
    b->cfg = *cfg;
    b->n = n;
    b->envs = (so_env **)calloc((size_t)n, sizeof *b->envs);
    if (!b->envs) { free(b); return NULL; }
    for (int64_t i = 0; i < n; i++) {
        if (!(b->envs[i] = so_create(cfg, seed + (uint32_t)i))) { so_batch_destroy(b); return NULL; }
    }
    b->obs_sz = so_obs_size(b->envs[0]);
    return b;
}

void so_batch_destroy(so_batch *b)
{
    if (!b) return;
    if (b->envs)
        for (int64_t i = 0; i < b->n; i++) if (b->envs[i]) so_destroy(b->envs[i]);
    free(b->envs);
    free(b);
}

typedef struct {
    so_batch *b;
    int64_t lo, hi;
    const int8_t *actions;      /* NULL: reset */
    uint8_t *obs, *dones, *ep_done;
    double *rews, *ep_stats;    /* ep_stats [n][4][S] */
    int32_t *rank, *err;
} so_batch_job;

static void *so_batch_run(void *arg)
{
    so_batch_job *j = (so_batch_job *)arg;
    const int S = j->b->cfg.num_snakes;
    for (int64_t i = j->lo; i < j->hi; i++) {
        so_env *e = j->b->envs[i];
        uint8_t *obs = j->obs + i * j->b->obs_sz;
        if (!j->actions) { so_reset(e, obs); continue; }
        int32_t a[16];
        for (int k = 0; k < S; k++) a[k] = j->actions[i * S + k];
        so_info info;
        memset(&info, 0, sizeof info);
        double *rw = j->rews + i * S;
        uint8_t *dn = j->dones + i * S;
        int32_t *rk = j->rank + i * S;
        double *es = j->ep_stats + i * 4 * S;
        int dir0[16];
        for (int k = 0; k < S; k++) dir0[k] = e->snakes[k].dir;
        const int rc = so_step(e, a, obs, rw, dn, &info);
        /* the reference turns the snakes before the invalid one, then raises;
         * the batch env (snake_env.h) leaves a rejected env entirely unchanged */
        if (rc < 0)
            for (int k = 0; k < S; k++) e->snakes[k].dir = dir0[k];
        j->ep_done[i] = rc == 1;
        j->err[i] = rc < 0;
        for (int k = 0; k < S; k++) {
            if (rc < 0) { rw[k] = 0.0; dn[k] = 0; }
            rk[k] = rc == 1 ? (int32_t)info.rank[k] : 0;
            es[k] = rc == 1 ? info.scores[k] : 0.0;
            es[S + k] = rc == 1 ? info.steps[k] : 0.0;
            es[2 * S + k] = rc == 1 ? info.fruits[k] : 0.0;
            es[3 * S + k] = rc == 1 ? info.kills[k] : 0.0;
        }
        if (rc < 0) emit_obs(e, obs);   /* rejected: the unchanged state's obs */
        if (rc == 1) so_reset(e, obs);
    }
    return NULL;
}

static int so_batch_launch(so_batch_job *proto, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 64) nthreads = 64;
    pthread_t th[64];
    so_batch_job jobs[64];
    const int64_t n = proto->b->n, per = (n + nthreads - 1) / nthreads;
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = *proto;
        jobs[t].lo = t * per < n ? t * per : n;
        jobs[t].hi = (t + 1) * per < n ? (t + 1) * per : n;
        if (t == 0) continue;
        if (pthread_create(&th[t], NULL, so_batch_run, &jobs[t]) != 0) {
            so_batch_run(&jobs[t]);   /* no thread: run it here */
            th[t] = 0;
        }
    }
    so_batch_run(&jobs[0]);
    for (int t = 1; t < nthreads; t++) if (th[t]) pthread_join(th[t], NULL);
    return 0;
}

int so_batch_reset(so_batch *b, uint8_t *obs, int nthreads)
{
    so_batch_job j;
    memset(&j, 0, sizeof j);
    j.b = b; j.obs = obs;
    return so_batch_launch(&j, nthreads);
}

int so_batch_step(so_batch *b, const int8_t *actions, uint8_t *obs, double *rews, uint8_t *dones,
                  uint8_t *ep_done, int32_t *rank, double *ep_stats, int32_t *err, int nthreads)
{
    so_batch_job j;
    memset(&j, 0, sizeof j);
    j.b = b; j.actions = actions; j.obs = obs; j.rews = rews; j.dones = dones; j.ep_done = ep_done;
    j.rank = rank; j.ep_stats = ep_stats; j.err = err;
    return so_batch_launch(&j, nthreads);
}

void so_batch_grids(const so_batch *b, uint8_t *out)
{
    const int64_t hw = (int64_t)b->cfg.height * b->cfg.width;
    for (int64_t i = 0; i < b->n; i++) so_get_grid(b->envs[i], out + i * hw);
}
