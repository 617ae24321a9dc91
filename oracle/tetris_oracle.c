/*
 * tetris_oracle.c -- CPU restatement of gym-simpletetris' step path.
 *
 * TEST INFRASTRUCTURE ONLY (see tetris_oracle.h).  Every function cites the
 * reference line it restates; paths are relative to /root/reference and
 * `tetris_env.py` = gym_simpletetris/envs/tetris_env.py.  The board is kept
 * as a byte array board[x][y] and pieces as 4 (dx,dy) cells exactly like the
 * reference, so this file checks the bit-packed HIP kernels independently.
 */
#include "tetris_oracle.h"
#include <string.h>

/* ------------------------------------------------------------------ */
/* CPython 3.10 random: Modules/_randommodule.c (MT19937, 2002 version) */
/* ------------------------------------------------------------------ */
#define MT_M 397
#define MT_MATRIX_A 0x9908b0dfU
#define MT_UPPER 0x80000000U
#define MT_LOWER 0x7fffffffU

static void mt_init_genrand(or_mt *m, uint32_t s) {
    m->mt[0] = s;
    for (int i = 1; i < OR_MT_N; i++)
        m->mt[i] = 1812433253U * (m->mt[i - 1] ^ (m->mt[i - 1] >> 30)) + (uint32_t)i;
    m->index = OR_MT_N;
}

static void mt_init_by_array(or_mt *m, const uint32_t *key, int len) {
    mt_init_genrand(m, 19650218U);
    int i = 1, j = 0;
    for (int k = (OR_MT_N > len ? OR_MT_N : len); k; k--) {
        m->mt[i] = (m->mt[i] ^ ((m->mt[i - 1] ^ (m->mt[i - 1] >> 30)) * 1664525U)) + key[j] + (uint32_t)j;
        i++; j++;
        if (i >= OR_MT_N) { m->mt[0] = m->mt[OR_MT_N - 1]; i = 1; }
        if (j >= len) j = 0;
    }
    for (int k = OR_MT_N - 1; k; k--) {
        m->mt[i] = (m->mt[i] ^ ((m->mt[i - 1] ^ (m->mt[i - 1] >> 30)) * 1566083941U)) - (uint32_t)i;
        i++;
        if (i >= OR_MT_N) { m->mt[0] = m->mt[OR_MT_N - 1]; i = 1; }
    }
    m->mt[0] = 0x80000000U;
}

/* random.seed(a) for int a >= 0: random_seed() splits abs(a) into 32-bit
 * little-endian limbs (key = [0] for a == 0) and calls init_by_array. */
void or_mt_seed_u64(or_mt *m, uint64_t seed) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    int len = (seed >> 32) ? 2 : 1;
    mt_init_by_array(m, key, len);
}

uint32_t or_mt_genrand(or_mt *m) {
    static const uint32_t mag01[2] = {0x0U, MT_MATRIX_A};
    uint32_t y;
    if (m->index >= OR_MT_N) {
        int kk;
        for (kk = 0; kk < OR_MT_N - MT_M; kk++) {
            y = (m->mt[kk] & MT_UPPER) | (m->mt[kk + 1] & MT_LOWER);
            m->mt[kk] = m->mt[kk + MT_M] ^ (y >> 1) ^ mag01[y & 1U];
        }
        for (; kk < OR_MT_N - 1; kk++) {
            y = (m->mt[kk] & MT_UPPER) | (m->mt[kk + 1] & MT_LOWER);
            m->mt[kk] = m->mt[kk + (MT_M - OR_MT_N)] ^ (y >> 1) ^ mag01[y & 1U];
        }
        y = (m->mt[OR_MT_N - 1] & MT_UPPER) | (m->mt[0] & MT_LOWER);
        m->mt[OR_MT_N - 1] = m->mt[MT_M - 1] ^ (y >> 1) ^ mag01[y & 1U];
        m->index = 0;
    }
    y = m->mt[m->index++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680U;
    y ^= (y << 15) & 0xefc60000U;
    y ^= (y >> 18);
    return y;
}

/* Lib/random.py:239-249 _randbelow_with_getrandbits; getrandbits(k<=32) is
 * genrand_uint32() >> (32 - k) (_randommodule.c _random_Random_getrandbits). */
uint32_t or_mt_randbelow(or_mt *m, uint32_t n) {
    if (!n) return 0;
    int k = 32 - __builtin_clz(n); /* n.bit_length() */
    uint32_t r = or_mt_genrand(m) >> (32 - k);
    while (r >= n) r = or_mt_genrand(m) >> (32 - k);
    return r;
}

/* ------------------------------------------------------------------ */
/* Engine: tetris_env.py                                              */
/* ------------------------------------------------------------------ */

/* tetris_env.py:10-19 -- shapes in shape_names order T,J,L,Z,S,I,O. */
static const int32_t k_shapes[7][4][2] = {
    {{0, 0}, {-1, 0}, {1, 0}, {0, -1}},   /* T */
    {{0, 0}, {-1, 0}, {0, -1}, {0, -2}},  /* J */
    {{0, 0}, {1, 0}, {0, -1}, {0, -2}},   /* L */
    {{0, 0}, {-1, 0}, {0, -1}, {1, -1}},  /* Z */
    {{0, 0}, {-1, -1}, {0, -1}, {1, 0}},  /* S */
    {{0, 0}, {0, -1}, {0, -2}, {0, -3}},  /* I */
    {{0, 0}, {0, -1}, {-1, 0}, {-1, -1}}, /* O */
};

/* tetris_env.py:22-26 rotated(shape, cclk). */
static void rotated(int32_t out[4][2], int32_t in[4][2], int cclk) {
    for (int c = 0; c < 4; c++) {
        int32_t i = in[c][0], j = in[c][1];
        if (cclk) { out[c][0] = -j; out[c][1] = i; }
        else      { out[c][0] = j;  out[c][1] = -i; }
    }
}

/* tetris_env.py:29-36 is_occupied. */
static int is_occupied(const or_env *e, int32_t shape[4][2], int32_t ax, int32_t ay) {
    for (int c = 0; c < 4; c++) {
        int32_t x = ax + shape[c][0], y = ay + shape[c][1];
        if (y < 0) continue;
        if (x < 0 || x >= e->cfg.width || y >= e->cfg.height || e->board[x][y]) return 1;
    }
    return 0;
}

/* tetris_env.py:39-73 the seven moves; each proposes and keeps the candidate
 * only if it is free.  Returns 1 if the piece moved/rotated. */
static void mv_translate(or_env *e, int32_t dx, int32_t dy) {
    if (!is_occupied(e, e->shape, e->ax + dx, e->ay + dy)) { e->ax += dx; e->ay += dy; }
}
static void mv_rotate(or_env *e, int cclk) {
    int32_t cand[4][2];
    rotated(cand, e->shape, cclk);
    if (!is_occupied(e, cand, e->ax, e->ay)) {
        memcpy(e->shape, cand, sizeof(cand));
        e->rot = (e->rot + (cclk ? 3 : 1)) & 3;
    }
}
static void mv_hard_drop(or_env *e) {            /* :54-59 */
    for (;;) {
        int32_t y0 = e->ay;
        mv_translate(e, 0, 1);
        if (e->ay == y0) return;
    }
}
/* value_action_map, :152-160. */
static void apply_action(or_env *e, int32_t a) {
    switch (a) {
    case 0: mv_translate(e, -1, 0); break;   /* left */
    case 1: mv_translate(e, 1, 0); break;    /* right */
    case 2: mv_hard_drop(e); break;          /* hard_drop */
    case 3: mv_translate(e, 0, 1); break;    /* soft_drop */
    case 4: mv_rotate(e, 0); break;          /* rotate_left: rotated(cclk=False) */
    case 5: mv_rotate(e, 1); break;          /* rotate_right: rotated(cclk=True) */
    default: break;                          /* idle */
    }
}

/* :183-191 _choose_shape: weights 5 + max(counts) - counts[i]. */
static int32_t choose_shape(or_env *e) {
    int32_t maxm = e->counts[0];
    for (int i = 1; i < 7; i++) if (e->counts[i] > maxm) maxm = e->counts[i];
    int32_t m[7], sum = 0;
    for (int i = 0; i < 7; i++) { m[i] = 5 + maxm - e->counts[i]; sum += m[i]; }
    int32_t r = 1 + (int32_t)or_mt_randbelow(&e->rng, (uint32_t)sum); /* randint(1, sum) */
    for (int i = 0; i < 7; i++) {
        r -= m[i];
        if (r <= 0) return i;
    }
    return 6; /* unreachable */
}

/* :193-200 _new_piece: anchor (width/2, 0); int() of it is width//2. */
static void new_piece(or_env *e) {
    e->ax = e->cfg.width / 2;
    e->ay = 0;
    e->shape_id = choose_shape(e);
    e->counts[e->shape_id] += 1;
    memcpy(e->shape, k_shapes[e->shape_id], sizeof(e->shape));
    e->rot = 0;
}

/* :323-327 _set_piece: paint cells that fall inside the board. */
static void set_piece(or_env *e, uint8_t on) {
    for (int c = 0; c < 4; c++) {
        int32_t x = e->ax + e->shape[c][0], y = e->ay + e->shape[c][1];
        if (x < e->cfg.width && x >= 0 && y < e->cfg.height && y >= 0) e->board[x][y] = on;
    }
}

/* :205-216 _clear_lines. */
static int32_t clear_lines(or_env *e) {
    const int32_t W = e->cfg.width, H = e->cfg.height;
    uint8_t can_clear[OR_MAX_H];
    int32_t n = 0;
    for (int y = 0; y < H; y++) {
        can_clear[y] = 1;
        for (int x = 0; x < W; x++) if (!e->board[x][y]) { can_clear[y] = 0; break; }
        n += can_clear[y];
    }
    uint8_t nb[OR_MAX_W][OR_MAX_H];
    memset(nb, 0, sizeof(nb));
    int32_t j = H - 1;
    for (int i = H - 1; i >= 0; i--) {
        if (!can_clear[i]) {
            for (int x = 0; x < W; x++) nb[x][j] = e->board[x][i];
            j--;
        }
    }
    e->lines_cleared += n;
    memcpy(e->board, nb, sizeof(nb));
    return n;
}

/* :218-220 _count_holes: count of (cumsum along y != 0) & cell empty. */
static int32_t count_holes(or_env *e) {
    int32_t holes = 0;
    for (int x = 0; x < e->cfg.width; x++) {
        int32_t cum = 0;
        for (int y = 0; y < e->cfg.height; y++) {
            cum += e->board[x][y];
            if (cum && !e->board[x][y]) holes++;
        }
    }
    e->holes = holes;
    return holes;
}

/* sum(np.any(board, axis=0)): number of non-empty rows, :287 / :289. */
static int32_t nonempty_rows(const or_env *e) {
    int32_t h = 0;
    for (int y = 0; y < e->cfg.height; y++) {
        for (int x = 0; x < e->cfg.width; x++) if (e->board[x][y]) { h++; break; }
    }
    return h;
}

void or_env_init(or_env *e, const or_config *cfg) {
    memset(e, 0, sizeof(*e));
    e->cfg = *cfg;
    e->time = -1;   /* :165 */
    e->score = -1;  /* :166 */
    memcpy(e->shape, k_shapes[0], sizeof(e->shape));
    or_mt_seed_u64(&e->rng, 0);
}

/* :306-315 clear(). n_deaths, shape_counts and _lock_delay persist. */
void or_env_clear(or_env *e) {
    e->time = 0;
    e->score = 0;
    e->holes = 0;
    e->lines_cleared = 0;
    e->piece_height = 0;
    new_piece(e);
    memset(e->board, 0, sizeof(e->board));
}

/* :243-304 step(). */
int32_t or_env_step(or_env *e, int32_t action, uint8_t *obs, int32_t *done_out, int32_t *rtype_out) {
    const or_config *c = &e->cfg;
    /* :244 anchor int cast is implicit (ints).  :245 action. */
    apply_action(e, action);
    /* :247-250 gravity */
    int32_t y0 = e->ay;
    mv_translate(e, 0, 1);
    if (c->step_reset && e->ay != y0) e->lock = 0;
    /* :253-256 */
    e->time += 1;
    int32_t reward = c->reward_step ? 1 : 0;
    int32_t rtype = OR_RT_INT;
    int32_t done = 0;
    /* :259 _has_dropped, :202-203 */
    if (is_occupied(e, e->shape, e->ax, e->ay + 1)) {
        e->lock = (e->lock + 1) % ((c->lock_delay > 0 ? c->lock_delay : 0) + 1); /* :175 */
        if (e->lock == 0) {
            set_piece(e, 1);                    /* :263 */
            int32_t n = clear_lines(e);         /* :264 */
            if (c->advanced_clears) {           /* :266-269 */
                static const int32_t scores[5] = {0, 40, 100, 300, 1200};
                reward += (scores[n] * 5) / 2;  /* 2.5 * scores[n], exact */
                e->score += scores[n];
                rtype = OR_RT_FLOAT;
            } else if (c->high_scoring) {       /* :270-272 */
                reward += 1000 * n;
                e->score += n;
                rtype = OR_RT_NP_INT64;
            } else {                            /* :273-275 */
                reward += 100 * n;
                e->score += n;
                rtype = OR_RT_NP_INT64;
            }
            int any_top = 0;                    /* :277 np.any(board[:, 0]) */
            for (int x = 0; x < c->width; x++) any_top |= e->board[x][0];
            if (any_top) {                      /* :277-281 */
                count_holes(e);
                e->n_deaths += 1;
                done = 1;
                reward = -100;
                rtype = OR_RT_INT;
            } else {
                int32_t old_holes = e->holes;   /* :283-284 */
                count_holes(e);
                if (c->penalise_height) {       /* :286-287 */
                    reward -= nonempty_rows(e);
                    if (rtype == OR_RT_FLOAT) rtype = OR_RT_NP_FLOAT64;
                } else if (c->penalise_height_increase) { /* :288-292 */
                    int32_t nh = nonempty_rows(e);
                    if (nh > e->piece_height) {
                        reward -= 10 * (nh - e->piece_height);
                        if (rtype == OR_RT_FLOAT) rtype = OR_RT_NP_FLOAT64;
                    }
                    e->piece_height = nh;
                }
                if (c->penalise_holes) reward -= 5 * e->holes;              /* :294-295 */
                else if (c->penalise_holes_increase) reward -= 5 * (e->holes - old_holes); /* :296-297 */
                new_piece(e);                   /* :299 */
            }
        }
    }
    /* :301-303 overlay, copy, erase */
    set_piece(e, 1);
    if (obs) {
        for (int x = 0; x < c->width; x++)
            for (int y = 0; y < c->height; y++) obs[x * c->height + y] = e->board[x][y];
    }
    set_piece(e, 0);
    if (done_out) *done_out = done;
    if (rtype_out) *rtype_out = rtype;
    return reward;
}

int32_t or_sizeof_env(void) { return (int32_t)sizeof(or_env); }

int64_t or_batch_rollout(or_env *envs, int32_t n, int32_t steps, const uint8_t *actions,
                         int32_t *rewards, uint8_t *dones, uint32_t *obs_cols, int32_t *stats) {
    int64_t locks = 0;
    uint8_t obs[OR_MAX_W * OR_MAX_H];
    for (int32_t t = 0; t < steps; t++) {
        for (int32_t i = 0; i < n; i++) {
            or_env *e = &envs[i];
            const int32_t W = e->cfg.width, H = e->cfg.height;
            int32_t done = 0, rtype = 0;
            int32_t before = 0;
            for (int k = 0; k < 7; k++) before += e->counts[k];
            int32_t r = or_env_step(e, actions[(int64_t)t * n + i], obs_cols ? obs : 0, &done, &rtype);
            int32_t after = 0;
            for (int k = 0; k < 7; k++) after += e->counts[k];
            locks += (after != before) || done;
            int64_t o = (int64_t)t * n + i;
            if (rewards) rewards[o] = r;
            if (dones) dones[o] = (uint8_t)done;
            if (obs_cols) {
                for (int x = 0; x < W; x++) {
                    uint32_t w = 0;
                    for (int y = 0; y < H; y++) w |= (uint32_t)obs[x * H + y] << y;
                    obs_cols[o * W + x] = w;
                }
            }
            if (stats) {
                int32_t *s = stats + o * 8;
                s[0] = e->time; s[1] = e->score; s[2] = e->lines_cleared; s[3] = e->holes;
                s[4] = e->n_deaths; s[5] = e->shape_id; s[6] = e->piece_height; s[7] = e->lock;
            }
            if (done) or_env_clear(e);
        }
    }
    return locks;
}
