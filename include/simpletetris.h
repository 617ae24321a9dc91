/*
 * simpletetris.h -- C ABI of the MI355X batched SimpleTetris step engine.
 *
 * This is the drop-in boundary for gym-simpletetris' per-step hot path.  The
 * reference has no FFI: its interface is the Python class
 * TetrisEnv/TetrisEngine in /root/reference/gym_simpletetris/envs/tetris_env.py.
 * Each entry point below names the reference method it replaces; the Python
 * host package (gym-simpletetris_amd/gym_simpletetris_amd) binds these with
 * ctypes and re-exposes the reference's Gym surface.
 *
 * Conventions
 *  - All functions return ST_OK (0) or a negative st_status; the message of
 *    the last failure on the calling thread is st_last_error().
 *  - Pointers named d_* are DEVICE pointers on the context's device; the
 *    caller owns them.  Context state (boards, pieces, counters, MT19937
 *    states) is owned by the context and lives in HBM.
 *  - Every call that takes a stream is asynchronous on that stream
 *    (NULL = the device's null stream).  Calls on one context must be
 *    serialised by the caller (the reference env is not thread-safe either,
 *    tetris_env.py:187 uses the global `random`).
 *  - Env e's piece RNG is CPython's MT19937 seeded with random.seed(seed[e]):
 *    results equal the reference run under the per-env isolation protocol
 *    (random.setstate/getstate around every reset/step of env e).
 */
#ifndef SIMPLETETRIS_H
#define SIMPLETETRIS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: st_step_wire carries the reward's 32 bits (st_wire_words grew by one
 * word for 10x20), st_unwire_shards.  3: st_gate_actions / st_gate_wait,
 * st_stream_wait (additions only).  4: st_step_n (addition only).
 * Snapshots (st_save) keep their own format version, unchanged. */
#define ST_ABI_VERSION 4

typedef struct st_ctx st_ctx;
typedef void *st_stream; /* hipStream_t */

typedef enum st_status {
    ST_OK = 0,
    ST_EINVAL = -1,  /* bad argument (reference: ValueError/KeyError) */
    ST_ENOMEM = -2,  /* device allocation failed */
    ST_EHIP = -3,    /* HIP runtime error */
    ST_ESTATE = -4   /* call order violated (e.g. step before seed) */
} st_status;

/* Scoring / rule flags: TetrisEngine.__init__ kwargs, tetris_env.py:126-137. */
enum st_flags {
    ST_REWARD_STEP = 1u << 0,               /* reward_step              :256 */
    ST_PENALISE_HEIGHT = 1u << 1,           /* penalise_height          :286 */
    ST_PENALISE_HEIGHT_INCREASE = 1u << 2,  /* penalise_height_increase :288 */
    ST_ADVANCED_CLEARS = 1u << 3,           /* advanced_clears          :266 */
    ST_HIGH_SCORING = 1u << 4,              /* high_scoring             :270 */
    ST_PENALISE_HOLES = 1u << 5,            /* penalise_holes           :294 */
    ST_PENALISE_HOLES_INCREASE = 1u << 6,   /* penalise_holes_increase  :296 */
    ST_STEP_RESET = 1u << 7                 /* step_reset               :248 */
};

/* What st_step does when an env dies (reference: the caller decides). */
enum st_autoreset {
    ST_AUTORESET_NONE = 0,     /* exact single-env semantics: state stays as the
                                  reference leaves it after a death step (incl.
                                  the R8 erase at tetris_env.py:303); caller
                                  calls st_reset(mask) like `if done: reset()` */
    ST_AUTORESET_SAME_STEP = 1 /* TetrisEngine.clear() runs inside the same
                                  kernel; obs is the terminal obs, terminal
                                  counters go to the ST_STAT_EP_* rows */
};

typedef struct st_config {
    int32_t width;      /* 4..32   (TetrisEnv width=10,  tetris_env.py:344) */
    int32_t height;     /* 4..28   (TetrisEnv height=20, tetris_env.py:345) */
    int32_t lock_delay; /* <= 32766 (tetris_env.py:356; negative acts as 0, :175) */
    uint32_t flags;     /* st_flags */
    int32_t autoreset;  /* st_autoreset */
} st_config;

/* Per-env int32 counters, SoA rows of the stats block (TetrisEngine.get_info,
 * tetris_env.py:232-241). */
enum st_stat {
    ST_STAT_TIME = 0,
    ST_STAT_SCORE = 1,
    ST_STAT_LINES = 2,
    ST_STAT_HOLES = 3,
    ST_STAT_PIECE_HEIGHT = 4,
    ST_STAT_DEATHS = 5,
    ST_STAT_COUNT0 = 6,   /* shape_counts T,J,L,Z,S,I,O: rows 6..12 */
    ST_STAT_MT_INDEX = 13,/* MT19937 index (0..624); see st_mt_sync */
    ST_STAT_PIECE = 14,   /* the piece word (uint32, = st_state_views.piece) */
    ST_STAT_EP_TIME = 15, /* terminal counters of the last finished episode */
    ST_STAT_EP_SCORE = 16,/* (ST_AUTORESET_SAME_STEP only)                   */
    ST_STAT_EP_LINES = 17,
    ST_STAT_EP_HOLES = 18,
    ST_NSTAT = 19
};

/* Device views of the context-owned state.  `stride` (>= n_envs, multiple of
 * 64) separates SoA rows.
 *   board  : uint32 [width][stride]  bit y of word (x, e) = board[x, y]
 *            (the reference's board[x, y], tetris_env.py:140, one bit-packed
 *            uint32 per board row x of the (width, height) array)
 *   piece  : uint32 [stride]  id | rot<<3 | anchor_x<<5 | anchor_y<<11 | lock<<17
 *            (an alias of stats row ST_STAT_PIECE)
 *            id in shape_names order T,J,L,Z,S,I,O (tetris_env.py:19);
 *            rot = number of rotate_left (rotated(cclk=False)) mod 4
 *   stats  : int32 [ST_NSTAT][stride]
 *   mt     : uint32 [stride][mt_pitch]; words [0, 624) of each row are the
 *            env's MT19937 state (CPython random.getstate()) after st_mt_sync;
 *            the rest is engine-private (the next generation, see st_mt_sync) */
typedef struct st_state_views {
    uint32_t *board;
    uint32_t *piece;
    int32_t *stats;
    uint32_t *mt;
    int64_t n_envs;
    int64_t stride;
    int32_t width, height;
    int64_t mt_pitch; /* words between consecutive envs' rows of mt */
} st_state_views;

/* ---- lifecycle: TetrisEnv.__init__ (tetris_env.py:343-392) ---------------- */
int st_create(st_ctx **out, const st_config *cfg, int device, int64_t n_envs); /* n_envs <= 2^24 */
int st_destroy(st_ctx *ctx);                     /* TetrisEnv.close, :466 */

/* random.seed(seed[e]) for every env (host array of n_envs uint64 seeds).
 * Also initialises counters as TetrisEngine.__init__ does (time = score = -1,
 * :165-166).  Required before the first st_reset. */
int st_seed(st_ctx *ctx, const uint64_t *seeds_host, st_stream stream);

/* TetrisEngine.clear (tetris_env.py:306-315) on every env with d_mask[e] != 0
 * (d_mask == NULL: all envs).  The reference's reset observation is the empty
 * board (clear() returns the board before the piece is drawn), so no
 * observation is produced here. */
int st_reset(st_ctx *ctx, const uint8_t *d_mask, st_stream stream);

/* TetrisEnv.step (tetris_env.py:397-403) / TetrisEngine.step (:243-304) on
 * every env.  d_actions: uint8 [n_envs] in 0..6 (values >= 7 are rejected on
 * the host side by the wrapper; the kernel treats them as idle).
 * Outputs (any may be NULL):
 *   d_obs    : uint32 [width][n_envs]  packed observation (board + current
 *              piece overlay, :301-302), same bit layout as st_state_views.board
 *   d_reward : int32 [n_envs]   (every reference reward is integer-valued)
 *   d_done   : uint8 [n_envs]                                                 */
int st_step(st_ctx *ctx, const uint8_t *d_actions, uint32_t *d_obs, int32_t *d_reward,
            uint8_t *d_done, st_stream stream);

/* Same as st_step but also writes the float32 observation the reference
 * returns (np.array(state, float32), :400): d_obs_f32 float [n_envs][width][height],
 * fused into the step kernel. */
int st_step_f32(st_ctx *ctx, const uint8_t *d_actions, uint32_t *d_obs, float *d_obs_f32,
                int32_t *d_reward, uint8_t *d_done, st_stream stream);

/* k consecutive steps (TetrisEngine.step k times, :243-304), one step
 * kernel launch each, enqueued by one host call: step i takes the actions at
 * device pointer d_actions[i] (d_actions: a HOST array of k device
 * pointers) and writes d_obs / d_obs_f32 (NULL: packed only) / d_reward /
 * d_done, so each holds step k-1's outputs when the stream reaches the end
 * -- st_step / st_step_f32 called k times, without the caller's per-call
 * host overhead between the launches (a native driver loop).  An armed
 * st_gate_actions gates the first of the k steps only.  k <= 0: nothing. */
int st_step_n(st_ctx *ctx, const uint8_t *const *d_actions, int64_t k, uint32_t *d_obs, float *d_obs_f32,
              int32_t *d_reward, uint8_t *d_done, st_stream stream);

/* st_step for a vector env (gym's autoreset convention), one
 * launch.  d_obs_f32 may be NULL (packed only).
 *   d_final_obs (uint32 [width][n_envs], or NULL): when given, an env that
 *     died and was reset inside this step (ST_AUTORESET_SAME_STEP) returns
 *     the RESET observation in d_obs / d_obs_f32 -- the empty board that
 *     clear() returns (tetris_env.py:306-315, :405-411) -- and its terminal
 *     observation (what the reference's step returned, :301-302) is written
 *     to d_final_obs.  Only the columns of such envs are meaningful (the
 *     kernel writes 16-B groups holding one).  NULL: the terminal obs is
 *     returned in d_obs (st_step's convention).  d_final_obs requires d_obs
 *     (ST_EINVAL otherwise).
 *   d_info (int32 [ST_NSTAT][n_envs], or NULL): every counter row after the
 *     step (get_info, :232-241, from one snapshot written by the step
 *     kernel): rows ST_STAT_* as in st_state_views.stats except
 *     ST_STAT_MT_INDEX (not written); the ST_STAT_EP_* rows hold the
 *     finished episode's counters where the env was reset in this step and
 *     0 elsewhere.
 * The headline st_step kernel is a separate instantiation: these outputs
 * cost it nothing. */
int st_step_vec(st_ctx *ctx, const uint8_t *d_actions, uint32_t *d_obs, float *d_obs_f32,
                int32_t *d_reward, uint8_t *d_done, uint32_t *d_final_obs, int32_t *d_info,
                st_stream stream);

/* BASELINE C5's gather format.  st_step_wire is st_step writing, instead of
 * obs / reward / done, one bit stream per env: column x's `height` obs bits
 * (exactly st_step's packed obs word x) at bit x*height, then the reward's
 * 32 bits (two's complement: lossless for every int32 the step computes,
 * host-written counters included) and the done bit -- stored as
 * st_wire_words(width, height) = ceil((width*height + 33) / 32) uint32 rows
 * d_wire [words][n_envs] (10x20: 8 words, 32 B per env, against 48 B for
 * obs + reward + done as width + 2 rows), so a per-step gather of every
 * shard's outputs to rank 0 (tetris_env.py:397-403's return values, for all
 * envs) moves 1.5x fewer bytes over xGMI.  st_unwire turns wire rows back
 * into st_step's outputs (d_obs uint32 [width][n], d_reward int32 [n],
 * d_done uint8 [n]), bit-exact.  st_unwire_shards does the same straight from
 * a gather's receive buffer: d_wire [shards][words][n_cap], shard r's envs at
 * its columns 0 .. count_r - 1, where shard r holds the contiguous global
 * block of distributed.shard_range (counts n_global / shards, the first
 * n_global % shards shards one more; n_cap >= the largest count) -> d_obs
 * [width][n_global], d_reward [n_global], d_done [n_global] in global env
 * order.  st_wire_words returns ST_EINVAL for a board outside 1..32 x 1..28. */
int st_wire_words(int32_t width, int32_t height);
int st_step_wire(st_ctx *ctx, const uint8_t *d_actions, uint32_t *d_wire, st_stream stream);
int st_unwire(int32_t width, int32_t height, int64_t n, const uint32_t *d_wire, uint32_t *d_obs,
              int32_t *d_reward, uint8_t *d_done, st_stream stream);
int st_unwire_shards(int32_t width, int32_t height, int64_t n_global, int32_t shards, int64_t n_cap,
                     const uint32_t *d_wire, uint32_t *d_obs, int32_t *d_reward, uint8_t *d_done,
                     st_stream stream);

/* k consecutive st_step calls in ONE launch: the driver loop of README.md:43-51
 * (`for t: obs, r, done, info = env.step(a[t])`) with all actions known up
 * front (synthetic / replayed rollouts).  Boards and counters stay on chip
 * between steps.  d_actions: uint8 [k][n_envs]; outputs per step at [t]
 * (any may be NULL): d_obs uint32 [k][width][n_envs], d_obs_f32 float
 * [k][n_envs][width][height], d_reward int32 [k][n_envs], d_done uint8
 * [k][n_envs].  Results are identical to k calls of st_step / st_step_f32. */
int st_rollout(st_ctx *ctx, int32_t k, const uint8_t *d_actions, uint32_t *d_obs,
               float *d_obs_f32, int32_t *d_reward, uint8_t *d_done, st_stream stream);

/* Packed obs (uint32 [width][n_envs]) -> float32 [n_envs][width][height]
 * (TetrisEnv._observation 'ram' + the float32 cast, :400 / :421-424). */
int st_obs_to_f32(st_ctx *ctx, const uint32_t *d_obs, float *d_out, st_stream stream);

/* TetrisEngine.render() (tetris_env.py:317-321): board with the current
 * piece overlaid, packed like st_step's d_obs (uint32 [width][n_envs]), for
 * every env, without stepping. */
int st_render(st_ctx *ctx, uint32_t *d_obs, st_stream stream);

/* Grayscale / RGB image of packed observations: convert_grayscale(board, size)
 * (tetris_env.py:76-114) [+ convert_grayscale_rgb, :117-122], evaluated in
 * closed form per pixel.  d_out: [n_envs][size][size][channels]
 * (channels 1 or 3), float32 (as_u8 == 0: TetrisEnv obs, :426-433) or uint8
 * (as_u8 != 0: render('rgb_array'), :458-462).  Values 0 / 128 / 190. */
int st_grayscale(st_ctx *ctx, const uint32_t *d_obs, int32_t size, int32_t channels,
                 int32_t as_u8, void *d_out, st_stream stream);

/* One env's step outputs and state as one record of st_export_words(width,
 * height) uint32 words, for the single-env surface's per-step read-back in
 * ONE transfer (TetrisEnv.step's obs / reward / done and get_info's counters,
 * tetris_env.py:397-403, :232-241, and CPython's random state, :187):
 *   [0, width)              packed obs word x of `env` (from d_obs [width][n_envs])
 *   width                   reward (from d_reward)      width + 1   done (d_done)
 *   width + 2 + r           stats row r, r < ST_NSTAT (ST_STAT_PIECE: the piece word)
 *   M + i, i < 624          (parts & ST_EXPORT_MT) MT word i, M = width + 2 + ST_NSTAT
 *   M + 624 + x*height + y  (parts & ST_EXPORT_OBS_F32) cell (x, y) of the obs
 *                           as float32 0.0 / 1.0: np.array(state, float32), :400
 * Parts not requested are not written.  d_obs / d_reward / d_done may be
 * NULL (zeros written).  The MT words and the ST_STAT_MT_INDEX word are
 * CPython's form (random.getstate(), as st_mt_sync would leave them) without
 * changing the env's state.  d_out: device memory (or host memory the device
 * can write). */
#define ST_EXPORT_MT 1u
#define ST_EXPORT_OBS_F32 2u
int st_export_env(st_ctx *ctx, int64_t env, const uint32_t *d_obs, const int32_t *d_reward,
                  const uint8_t *d_done, uint32_t parts, uint32_t *d_out, st_stream stream);
int st_export_words(int32_t width, int32_t height);

/* Device views of the state (valid until st_destroy). */
int st_state(st_ctx *ctx, st_state_views *out);

/* hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, stream) -- moves state
 * between the views above and caller buffers (crafted states). */
int st_copy(void *dst, const void *src, int64_t bytes, st_stream stream);

/* The step kernels keep each env's MT19937 generation double-buffered (the
 * next generation is computed a few words per draw into a second buffer and
 * becomes current at index 624) and draw every env's next piece one spawn
 * ahead (the "preview", whose words the reference has not consumed yet), so
 * between steps ST_STAT_MT_INDEX carries engine bits above bit 9 and the
 * current words may sit in the second buffer.  st_mt_sync (on `stream`)
 * brings every env back to CPython's form -- words [0, 624) of its mt row and
 * an index 0..624 equal random.getstate(), the preview's words given back.
 * Call it before reading stats or mt through st_state's views; st_save calls
 * it itself.  Writing a CPython state (words [0, 624), index 0..624) is always
 * valid. */
int st_mt_sync(st_ctx *ctx, st_stream stream);

/* State snapshot: the engine attributes of every env (board, piece, counters,
 * shape counts: TetrisEngine.__init__ / _new_piece, tetris_env.py:138-199)
 * and its MT19937 state (CPython random.getstate(), :187).
 * st_state_bytes: the size of one snapshot of this context.
 * st_save: writes it to host memory (a 64-byte header -- magic "STSNAP\0\1",
 *   snapshot format version (1), width, height, ST_NSTAT, n_envs -- then board uint32
 *   [width][n_envs], stats int32 [ST_NSTAT][n_envs], mt uint32 [n_envs][624]).
 * st_load: restores one into a context with the same width, height and
 *   n_envs (scoring flags and lock delay are configuration, not state, and
 *   may differ).  A loaded context needs no st_seed / st_reset.
 * Both synchronous; ST_EINVAL on a size or header mismatch. */
int64_t st_state_bytes(const st_ctx *ctx);
int st_save(st_ctx *ctx, void *host_out, int64_t bytes);
int st_load(st_ctx *ctx, const void *host_in, int64_t bytes);

/* Greedy placement policy (a benchmark / test workload generator, not part
 * of the reference env; SURVEY 8(d) "clear-heavy variant"): d_actions[e] =
 * the action a greedy player takes in env e's current state -- rotate_left
 * toward, then move toward, then hard-drop onto the placement maximizing
 * 80*lines - 12*holes - 3*height - 2000*(piece above the top) over all
 * (rotation, anchor x) hard-dropped from row 0 (first maximum in rotation,
 * then x order) -- or, with probability explore_permille/1000, the uniform
 * action splitmix64(seed ^ ((t << 32) ^ e)) >> 32 mod 7.  Reads the state
 * enqueued before it on `stream`. */
int st_policy_greedy(st_ctx *ctx, uint64_t seed, int64_t t, uint32_t explore_permille,
                     uint8_t *d_actions, st_stream stream);

/* Synthetic action source used by the benchmark and the parity tests:
 * d_out[e] = splitmix64(seed ^ ((t << 32) ^ (global_offset + e))) % 7. */
int st_gen_actions(uint8_t *d_out, int64_t n, int64_t t, uint64_t seed,
                   int64_t global_offset, st_stream stream);

/* Sticky check for actions outside 0..6 (the reference raises KeyError for
 * them, tetris_env.py:245; st_step treats them as idle) as its own launch,
 * for an action batch not (yet) passed to a step: sets *d_flag = 1 if
 * any of d_actions[0..n) is > 6, never clears it.  d_flag may be host memory
 * mapped for the device, so the caller can poll it without synchronising
 * (the batched surface's validate_actions='async'). */
int st_check_actions(const uint8_t *d_actions, int64_t n, uint32_t *d_flag, st_stream stream);

/* The same check fused into the step kernels: once a flag word is set,
 * every st_step / st_step_f32 / st_rollout on this context sets *d_flag = 1
 * when any of its actions is > 6 (never clears it), from the action loads the
 * step does anyway -- no extra launch, no sync.  d_flag: device memory or host
 * memory mapped for the device (st_host_device_ptr), owned by the caller and
 * valid until it is replaced; NULL turns the check off (the default). */
int st_set_action_flag(st_ctx *ctx, uint32_t *d_flag);

/* The reference's immediate KeyError (tetris_env.py:245: value_action_map
 * [action] fails before TetrisEngine.step changes any state) for actions
 * already on the device, without draining the stream:
 *   st_gate_actions checks d_actions[0..n_envs) on `stream` (one small
 *     launch) and records an event behind it; the NEXT st_step / st_step_f32 /
 *     st_step_vec on this context is gated: if any action was outside 0..6 it
 *     changes no env and writes no output (every env is skipped), else it is
 *     the ordinary step.  Enqueue that step right away.
 *   st_gate_wait then waits for the check only (the event; the gated step is
 *     already queued behind it and runs while the host waits) and returns 1 if
 *     an action was outside 0..6 (the step was skipped: raise KeyError), 0 if
 *     not, < 0 on error (ST_ESTATE without a pending st_gate_actions).
 * Other calls (st_step_wire, st_rollout, st_reset) are not gated and do not
 * consume the gate. */
int st_gate_actions(st_ctx *ctx, const uint8_t *d_actions, st_stream stream);
int st_gate_wait(st_ctx *ctx);

/* Runtime helpers for hosts that bind only this library (the Python package
 * uses them instead of opening the HIP runtime by name, which could load a
 * second runtime copy beside the one the kernels use):
 * st_stream_sync: hipStreamSynchronize(stream);
 * st_host_device_ptr: the device address of pinned, mapped host memory
 * (hipHostGetDevicePointer);
 * st_stream_wait: work enqueued on `waiter` after this call waits (on the
 * device, no host wait) for the work enqueued on `signaller` before it
 * (hipEventRecord + hipStreamWaitEvent; both streams on the current device).
 * The vector env orders its reuse of an output slot behind the consumer
 * streams a caller registered (TetrisVecEnv.record_stream). */
int st_stream_sync(st_stream stream);
int st_host_device_ptr(void *host, void **d_out);
int st_stream_wait(st_stream waiter, st_stream signaller);

/* Diagnostics: when the environment variable ST_STAMPS is set at st_create,
 * st_step runs an instrumented build of the step kernel that records
 * s_memtime at its phase boundaries per wave; this copies the last step's
 * stamps ([n_waves][16] uint64: 10 phase stamps, s_memrealtime at start and
 * end, HW_ID, XCC_ID) to host memory.  Timing study only. */
int st_debug_stamps(st_ctx *ctx, uint64_t *host_out, int64_t max_words);

/* Message for the last failed call on this thread ("" if none). */
const char *st_last_error(void);
int st_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* SIMPLETETRIS_H */
