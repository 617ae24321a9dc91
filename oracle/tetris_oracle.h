/*
 * tetris_oracle.h -- CPU restatement of gym-simpletetris' step path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle: a plain-C,
 * cell-by-cell restatement of /root/reference/gym_simpletetris/envs/tetris_env.py
 * (TetrisEngine, lines 125-335) plus CPython 3.10's `random` module
 * (MT19937 + randint), which the reference uses for piece selection.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it.  The shipped product (gym-simpletetris_amd/) never links it.
 *
 * Parity pin: tests/golden/ fixtures, generated in the build container by
 * importing the reference itself (tests/golden/gen_golden.py), plus
 * MT19937 known-answer vectors produced by CPython's own `random`.
 */
#ifndef TETRIS_ORACLE_H
#define TETRIS_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OR_MAX_W 32
#define OR_MAX_H 32
#define OR_MT_N 624

/* CPython _randommodule.c RandomObject state. */
typedef struct {
    uint32_t mt[OR_MT_N];
    int32_t index;
} or_mt;

/* TetrisEngine.__init__ kwargs, tetris_env.py:126-137. */
typedef struct {
    int32_t width, height, lock_delay, step_reset;
    int32_t reward_step, penalise_height, penalise_height_increase;
    int32_t advanced_clears, high_scoring, penalise_holes, penalise_holes_increase;
} or_config;

/* One TetrisEngine instance (tetris_env.py:138-181) + its private RNG. */
typedef struct {
    or_config cfg;
    uint8_t board[OR_MAX_W][OR_MAX_H]; /* board[x][y], :140 */
    int32_t shape[4][2];               /* current cells (i, j), :200 */
    int32_t shape_id;                  /* index into shape_names, :19 */
    int32_t rot;                       /* number of rotate_left applied mod 4 (bookkeeping only) */
    int32_t ax, ay;                    /* anchor, :196 / :244 */
    int32_t lock;                      /* _lock_delay, :176 */
    int32_t time, score, holes, lines_cleared, piece_height, n_deaths;
    int32_t counts[7];                 /* shape_counts, :181 */
    or_mt rng;
} or_env;

/* Reward python-type codes (reference R18): what type(reward) is. */
enum { OR_RT_INT = 0, OR_RT_NP_INT64 = 1, OR_RT_FLOAT = 2, OR_RT_NP_FLOAT64 = 3 };

/* ---- CPython random (Lib/random.py + Modules/_randommodule.c) ---- */
void or_mt_seed_u64(or_mt *m, uint64_t seed);          /* random.seed(int) */
uint32_t or_mt_genrand(or_mt *m);                      /* getrandbits(32) */
uint32_t or_mt_randbelow(or_mt *m, uint32_t n);        /* _randbelow_with_getrandbits */

/* ---- engine ---- */
void or_env_init(or_env *e, const or_config *cfg);
void or_env_clear(or_env *e);                          /* TetrisEngine.clear, :306 */
/* TetrisEngine.step, :243-304.  obs: W*H bytes board[x][y] with piece overlay.
 * Returns reward (all reference rewards are integer-valued). */
int32_t or_env_step(or_env *e, int32_t action, uint8_t *obs, int32_t *done, int32_t *rtype);

/* ---- batched helpers (tests / cpu baseline) ---- */
int32_t or_sizeof_env(void);
/* Steps `n` independent envs through `steps` steps with actions[t*n+e];
 * after a done the env is reset (reference driver: `if done: env.reset()`).
 * Any output pointer may be NULL.  obs_cols: packed column words
 * [t][e][x] (bit y of column x).  Returns total locks. */
int64_t or_batch_rollout(or_env *envs, int32_t n, int32_t steps, const uint8_t *actions,
                         int32_t *rewards, uint8_t *dones, uint32_t *obs_cols,
                         int32_t *stats /* [t][e][8]: time,score,lines,holes,deaths,piece,height,lock */);

#ifdef __cplusplus
}
#endif
#endif
