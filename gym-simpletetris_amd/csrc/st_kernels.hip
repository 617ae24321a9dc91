// st_kernels.hip -- MI355X (gfx950) kernels of the batched SimpleTetris engine.
//
// Hot path: TetrisEngine.step (/root/reference/gym_simpletetris/envs/tetris_env.py:243-304)
// for N independent envs, one env per lane, one wave (64 envs) per workgroup.
//
// Data layout (HBM, SoA over envs, row stride = padded env count):
//   board  u32 [W][stride]  bit y of word (x, e) = board[x, y]  (the reference's
//          (width, height) array, tetris_env.py:140, one bit-packed u32 per x)
//   piece  u32 [stride]     id | rot<<3 | ax<<5 | ay<<11 | lock<<17
//   stats  i32 [ST_NSTAT][stride]
//   mt     u32 [stride][624] per-env CPython MT19937 words (env-contiguous so a
//          wave can twist one env's state with coalesced 256-B accesses)
// Every load a step needs is issued up front (coalesced, 4 B/lane); the board
// is then staged into LDS as L[(x + kPad) * 64 + lane], which makes every
// per-lane dynamically indexed column access bank-conflict free (bank = lane).
// The column words carry "floor" bits at rows >= H and the kPad columns on
// each side are all-ones walls, so a collision test is four AND-tests with no
// bounds checks and hard_drop is a count-trailing-zeros per piece column.
#include "st_internal.h"


namespace st {
namespace {

// ---------------------------------------------------------------- pieces
// tetris_env.py:10-19, shape_names order T,J,L,Z,S,I,O.
constexpr int kShapes[7][4][2] = {
    {{0, 0}, {-1, 0}, {1, 0}, {0, -1}},   {{0, 0}, {-1, 0}, {0, -1}, {0, -2}},
    {{0, 0}, {1, 0}, {0, -1}, {0, -2}},   {{0, 0}, {-1, 0}, {0, -1}, {1, -1}},
    {{0, 0}, {-1, -1}, {0, -1}, {1, 0}},  {{0, 0}, {0, -1}, {0, -2}, {0, -3}},
    {{0, 0}, {0, -1}, {-1, 0}, {-1, -1}},
};

// One descriptor per (piece, rot) = {m, g}, four column records each:
//   m: byte j = the column's cells as a bit mask biased by 3 (bit dy+3);
//   g: 6 bits per column j: dx+3 (bits 6j..6j+2), bottom dy+3 (6j+3..6j+5).
// Tetromino columns are vertically contiguous runs (checked below); pieces
// with fewer than 4 columns repeat their last column (OR/AND/min idempotent).
// rot r = r applications of rotated(cclk=False) (tetris_env.py:22-26).
struct PieceTab {
    uint32_t m[28], g[28];
    bool ok;
};

constexpr PieceTab make_piece_tab() {
    PieceTab t{};
    t.ok = true;
    for (int p = 0; p < 7; ++p) {
        int cx[4] = {}, cy[4] = {};
        for (int c = 0; c < 4; ++c) {
            cx[c] = kShapes[p][c][0];
            cy[c] = kShapes[p][c][1];
        }
        for (int r = 0; r < 4; ++r) {
            uint32_t m = 0, g = 0, lm = 0, lg = 0;
            int ncol = 0;
            for (int dx = -3; dx <= 3; ++dx) {
                int ymin = 99, ymax = -99, cnt = 0;
                uint32_t bits = 0;
                for (int c = 0; c < 4; ++c)
                    if (cx[c] == dx) {
                        ++cnt;
                        ymin = cy[c] < ymin ? cy[c] : ymin;
                        ymax = cy[c] > ymax ? cy[c] : ymax;
                        bits |= 1u << (cy[c] + 3);
                    }
                if (!cnt) continue;
                if (cnt != ymax - ymin + 1 || ymin < -3 || ymax > 3) t.ok = false;
                lm = bits;
                lg = (uint32_t)(dx + 3) | ((uint32_t)(ymax + 3) << 3);
                m |= lm << (8 * ncol);
                g |= lg << (6 * ncol);
                ++ncol;
            }
            for (int j = ncol; j < 4; ++j) {
                m |= lm << (8 * j);
                g |= lg << (6 * j);
            }
            t.m[p * 4 + r] = m;
            t.g[p * 4 + r] = g;
            for (int c = 0; c < 4; ++c) {  // rotated(cclk=False): (i, j) -> (j, -i)
                const int i = cx[c], j = cy[c];
                cx[c] = j;
                cy[c] = -i;
            }
        }
    }
    return t;
}
constexpr PieceTab kTab = make_piece_tab();
static_assert(kTab.ok, "every tetromino column must be a contiguous run within [-3, 3]");
#define ST_TAB28(a) {a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7], a[8], a[9], a[10], a[11], \
                     a[12], a[13], a[14], a[15], a[16], a[17], a[18], a[19], a[20], a[21], a[22], \
                     a[23], a[24], a[25], a[26], a[27]}
__constant__ uint32_t c_tab_m[28] = ST_TAB28(kTab.m);
__constant__ uint32_t c_tab_g[28] = ST_TAB28(kTab.g);

// The rollout's piece table ("box columns"): a rotation's columns as four
// consecutive board columns from its leftmost, dx0 = (g & 7) - 3 (at most 0:
// every shape holds its anchor cell), column c's cells in byte c of m (0:
// none) and, in bits [3 + 7c, 10 + 7c) of g as a signed field, the row
// below its lowest cell relative to the anchor (bottom dy + 1; -64 for no
// cells: a bottom far above the board, which never stops a drop, see
// drop_box).  One address per descriptor: the four column reads take
// immediate offsets.
constexpr PieceTab make_box_tab() {
    PieceTab t{};
    t.ok = true;
    for (int p = 0; p < 7; ++p) {
        int cx[4] = {}, cy[4] = {};
        for (int c = 0; c < 4; ++c) {
            cx[c] = kShapes[p][c][0];
            cy[c] = kShapes[p][c][1];
        }
        for (int r = 0; r < 4; ++r) {
            int dx0 = 99, dx1 = -99;
            for (int c = 0; c < 4; ++c) {
                dx0 = cx[c] < dx0 ? cx[c] : dx0;
                dx1 = cx[c] > dx1 ? cx[c] : dx1;
            }
            if (dx0 < -3 || dx0 > 0 || dx1 - dx0 > 3) t.ok = false;
            uint32_t m = 0, g = (uint32_t)(dx0 + 3);
            for (int k = 0; k < 4; ++k) g |= 64u << (3 + 7 * k);
            for (int k = 0; k < 4; ++k) {
                int ymin = 99, ymax = -99, cnt = 0;
                uint32_t bits = 0;
                for (int c = 0; c < 4; ++c)
                    if (cx[c] == dx0 + k) {
                        ++cnt;
                        ymin = cy[c] < ymin ? cy[c] : ymin;
                        ymax = cy[c] > ymax ? cy[c] : ymax;
                        bits |= 1u << (cy[c] + 3);
                    }
                if (!cnt) continue;
                if (cnt != ymax - ymin + 1 || ymin < -3 || ymax > 3) t.ok = false;
                m |= bits << (8 * k);
                g = (g & ~(127u << (3 + 7 * k))) | ((uint32_t)(ymax + 1) & 127u) << (3 + 7 * k);
            }
            t.m[p * 4 + r] = m;
            t.g[p * 4 + r] = g;
            for (int c = 0; c < 4; ++c) {  // rotated(cclk=False): (i, j) -> (j, -i)
                const int i = cx[c], j = cy[c];
                cx[c] = j;
                cy[c] = -i;
            }
        }
    }
    return t;
}
constexpr PieceTab kBox = make_box_tab();
static_assert(kBox.ok, "every rotation must span at most four columns from dx0 in [-3, 0]");

// Column j of a descriptor: dx, bottom dy, and its cells at anchor row y as
// board-row bits; cells with y < 0 vanish (is_occupied skips them,
// tetris_env.py:32-33; _set_piece clips them, :326).
__device__ __forceinline__ int pc_dx(uint32_t g, int j) { return (int)((g >> (6 * j)) & 7u) - 3; }
__device__ __forceinline__ int pc_bot(uint32_t g, int j) { return (int)((g >> (6 * j + 3)) & 7u) - 3; }
// S32: board height <= 25 (compile time), so a cell's bit (row + 3 <= 30)
// fits a 32-bit shift.  (The 64-bit form's don't-care high half can land in
// a register still waiting on a load -- measured: the lock path's paint
// waited for the MT prefetch -- so the 32-bit form is used wherever it is
// exact.)
template <bool S32 = false>
__device__ __forceinline__ uint32_t pc_bits(uint32_t m, int j, int y) {
    if constexpr (S32) return (((m >> (8 * j)) & 0xFFu) << y) >> 3;
    return (uint32_t)((uint64_t)((m >> (8 * j)) & 0xFFu) << y >> 3);
}

// Branch-free masked stores: raw buffer stores whose lanes get an offset past
// the resource's range are dropped by the hardware (no traffic), and unlike a
// store under `if` they keep the compiler's vmcnt bookkeeping exact (a store
// skipped on some path turns later waits on older loads into vmcnt(0)).
typedef int i32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kOff = 0xFFFFFFF0u;  // "no store" offset (>= every range used)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void *base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, base ? (int)bytes : 0,
                                             0x00020000);
}
// Cache policy of the step's stores: non-temporal (gfx950 `nt`).  Lines a
// store leaves dirty in L2 are written back at the kernel's end, on the
// dependent launch's critical path (the guide's boundary cost + B / 6 TB/s);
// `nt` stores stream out during the kernel instead (A/B, st_step packed:
// 6.31 -> 5.89 us with obs, board, counter and MT stores all `nt`).
// (round 5, profiles/r05/ab_store_cache_policy.txt: `sc1` write-through
// +12..15%, `sc1 nt` +15%; the state stores alone write-back or `sc0` +1..2%,
// ab_state_store_cache_policy.txt)
constexpr int kNT = 2;
constexpr int kST = kNT;  // the state stores (board, counter rows, MT words)
// the reward / done stores: nt like the obs (round 5 A/B against the
// default policy, profiles/r05/ab_reward_done_nt.txt: -0.4..-0.9%)
constexpr int kRD = kNT;
// Wave issue priorities (s_setprio), settled by A/B in rounds 1-3:
// the draw wave after B1 at 2 (its chain was the critical one there: st_step
// -1.5%, rollouts -6%; 0 / 1 / 3 re-checked in round 3 within noise,
// profiles/r03/ab_step_prio.txt); st_step's logic wave at 1 from its first
// instruction (since the draw parameters moved before B1 its chain is the
// step: K = 2,000 4.67-4.72 -> 4.64-4.67 us, profiles/r03/ab_step_lprio.txt).
constexpr int kDrawPrio = 2;
constexpr int kLogicPrio = 1;
template <int AUX = 0>
__device__ __forceinline__ void buf_store16(__amdgpu_buffer_rsrc_t r, uint32_t off, uint4 v) {
    const i32x4 d = {(int)v.x, (int)v.y, (int)v.z, (int)v.w};
    __builtin_amdgcn_raw_buffer_store_b128(d, r, off, 0, AUX);
}

__device__ __forceinline__ uint32_t &lcol(uint32_t *L, int x, int lane) {
    return L[(x + kPad) * kWave + lane];
}

// The four column words a descriptor touches at anchor column x (issued as
// one batch of LDS reads), and the collision / drop tests on them:
//  collides_v = is_occupied (tetris_env.py:29-36) with the floor bits and the
//    all-ones wall columns standing in for the bounds checks; cells with y < 0
//    vanish in pc_bits (R2);
//  drop_v = the number of free soft_drops below a legal position, i.e.
//    hard_drop's loop count (tetris_env.py:54-59): only each column's lowest
//    cell can meet an obstacle first, and the first obstacle row is the lowest
//    set bit of (column | floor) at or below it.  A column outside the board
//    (legal only while its cells are above row 0) reads a wall and stops the
//    piece as its lowest cell would enter row 0.
__device__ __forceinline__ void read_cols(const uint32_t *L, int lane, uint32_t g, int x,
                                          uint32_t (&v)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = L[(x + pc_dx(g, j) + kPad) * kWave + lane];
}
template <bool S32 = false>
__device__ __forceinline__ bool collides_v(uint32_t m, int y, const uint32_t (&v)[4]) {
    uint32_t hit = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) hit |= pc_bits<S32>(m, j, y) & v[j];
    return hit != 0;
}
__device__ __forceinline__ int drop_v(uint32_t g, int y, const uint32_t (&v)[4]) {
    int dist = 1 << 20;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int yb = y + pc_bot(g, j);
        const int s = yb + 1 > 0 ? yb + 1 : 0;
        const int k = __builtin_ctz(v[j] & (~0u << s)) - yb - 1;
        dist = k < dist ? k : dist;
    }
    return dist;
}

// _set_piece(True) (tetris_env.py:323-327): cells inside the board only,
// as no-return LDS atomics.
template <bool S32 = false>
__device__ __forceinline__ void paint(uint32_t *L, int lane, uint32_t m, uint32_t g, int x, int y,
                                      uint32_t hmask) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
        atomicOr(&L[(x + pc_dx(g, j) + kPad) * kWave + lane], pc_bits<S32>(m, j, y) & hmask);  // ds_or_b32
}

// _set_piece(False): erase the cells.
template <bool S32 = false>
__device__ __forceinline__ void erase(uint32_t *L, int lane, uint32_t m, uint32_t g, int x, int y,
                                      uint32_t hmask) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
        atomicAnd(&L[(x + pc_dx(g, j) + kPad) * kWave + lane], ~(pc_bits<S32>(m, j, y) & hmask));
}

// Box-column forms of read_cols / drop_v / paint / erase (kBox descriptors).
// drop_box: q = the row below the column's lowest cell; a column without
// cells has q = y - 64, so its shift is 0 and its distance ctz(column) + 64
// - y exceeds every real column's (at most H + 2 - y: the floor bits stop a
// drop by row H < 32; every column word holds floor or wall bits, so ctz
// sees a set bit).  7 VALU a column, the first column seeding the minimum.
__device__ __forceinline__ int box_x0(uint32_t g, int x) { return x + (int)(g & 7u) - 3; }
__device__ __forceinline__ void read_box(const uint32_t *L, int lane, uint32_t g, int x, uint32_t (&v)[4]) {
    const uint32_t *c0 = &L[(box_x0(g, x) + kPad) * kWave + lane];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = c0[j * kWave];
}
__device__ __forceinline__ int drop_box(uint32_t g, int y, const uint32_t (&v)[4]) {
    int dist = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int q = y + ((int32_t)(g << (32 - 10 - 7 * j)) >> 25);  // v_bfe_i32
        const int s = q > 0 ? q : 0;
        const int k = __builtin_ctz(v[j] & (~0u << s)) - q;
        dist = j == 0 || k < dist ? k : dist;
    }
    return dist;
}
template <bool S32 = false>
__device__ __forceinline__ void paint_box(uint32_t *L, int lane, uint32_t m, uint32_t g, int x, int y,
                                          uint32_t hmask) {
    uint32_t *c0 = &L[(box_x0(g, x) + kPad) * kWave + lane];
#pragma unroll
    for (int j = 0; j < 4; ++j) atomicOr(&c0[j * kWave], pc_bits<S32>(m, j, y) & hmask);  // ds_or_b32
}
template <bool S32 = false>
__device__ __forceinline__ void erase_box(uint32_t *L, int lane, uint32_t m, uint32_t g, int x, int y,
                                          uint32_t hmask) {
    uint32_t *c0 = &L[(box_x0(g, x) + kPad) * kWave + lane];
#pragma unroll
    for (int j = 0; j < 4; ++j) atomicAnd(&c0[j * kWave], ~(pc_bits<S32>(m, j, y) & hmask));
}

// _clear_lines row compaction (tetris_env.py:205-216) on one column word:
// remove every row in `full` (processed top-down) and let the rows above fall.
__device__ __forceinline__ uint32_t compact(uint32_t v, uint32_t full) {
    while (full) {
        const int r = __builtin_ctz(full);
        full &= full - 1u;
        const uint32_t above = (1u << r) - 1u;
        v = (v & ~(above | (1u << r))) | ((v & above) << 1);
    }
    return v;
}

// Every kernel below that exchanges data between lanes through LDS runs one
// wave per workgroup.  LDS operations of a wavefront execute in order, so a
// read issued after another lane's write returns that write's data: the
// exchange needs only compiler ordering, not __syncthreads' full
// s_waitcnt lgkmcnt(0) (which would stall the wave for each LDS round trip).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---------------------------------------------------------------- MT19937
// CPython Modules/_randommodule.c genrand_uint32 / init_by_array.
__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    // y ^ (t & B) as one v_bitop3 (truth table 0x78 = a ^ (b & c) with the
    // a=0xF0 / b=0xCC / c=0xAA convention)
    y ^= (y >> 11);
    y = __builtin_amdgcn_bitop3_b32(y, y << 7, 0x9d2c5680u, 0x78);
    y = __builtin_amdgcn_bitop3_b32(y, y << 15, 0xefc60000u, 0x78);
    y ^= (y >> 18);
    return y;
}
// The tempering without its last step (y ^= y >> 18), which changes bits < 14
// only: the top 18 bits of the result are exact.
__device__ __forceinline__ uint32_t mt_temper_hi18(uint32_t y) {
    y ^= (y >> 11);
    y = __builtin_amdgcn_bitop3_b32(y, y << 7, 0x9d2c5680u, 0x78);
    return __builtin_amdgcn_bitop3_b32(y, y << 15, 0xefc60000u, 0x78);
}
__device__ __forceinline__ uint32_t mt_mix(uint32_t a, uint32_t b) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

// ---- Double-buffered twist --------------------------------------------------
// CPython refills its 624 words at once when the index reaches 624:
//   new[k] = X_k ^ mix(old[k], old[k+1]),  X_k = old[k+397] (k < 227) | new[k-227] (k >= 227),
//   new[623] = new[396] ^ mix(old[623], new[0]).
// Each env keeps two generation buffers A and B (kMtPitch words: A[624] B[624]
// pad[16]).  Draws read the current one; the next generation is computed into
// the other, 64 words at a time: once per step every wave builds one 64-word
// chunk of ONE of its envs' next generations (mt_chunk_*: the lowest lane
// whose successor is incomplete), one word per lane, with coalesced 256-B
// loads and stores -- 10 chunks per generation.  A draw uses 1/P(accept) <= 2
// words on average, so a generation lasts >= ~312 draws (~1,500 steps at the
// uniform-action lock rate); its wave has a chunk slot every step, and 64
// envs x 10 chunks per ~1,500 steps use under half of them.  The switch at
// index 624 is then a bit flip, and no wave runs the 624-word twist on the
// hot path (eagerly, a twisting wave took ~16k cycles, 2x the others, and set
// the step's length whenever one occurred).  (Round 1 built one 4-word block
// per locking lane instead: its operand loads touched ~3 cache lines per
// lock for ~36 bytes used.)  A successor not ready in time (a host-written or
// synced state restarts the progress at 0) is finished wave-cooperatively
// (mt_finish).
//
// Layout: cur[624..639] is next[0..15] for both parities -- B[0..15] for cur
// = A; the pad, which the writers of A[0..15] also fill, for cur = B -- so a
// block's operands cur[p..p+4] and cur[p+397..p+400] (p <= 224; X_227 =
// new[0]) need no case split, neither does new[623]'s mix(old[623], new[0]),
// and a draw window that runs past 623 continues into a complete successor.
//
// State (stats row ST_STAT_MT_INDEX): idx | p << 10 | cur << 20
//   idx: CPython's index into the current buffer (0..624)
//   p  : words of the next generation done (0..624; a multiple of 4 unless
//        624: chunks start at any multiple of 4 a host state or mt_finish left)
//   cur: 0 = A, 1 = B.
// A host-written CPython index (p = cur = 0, state in A) is always valid;
// st_mt_sync (k_mt_sync) brings every env back to that form.
constexpr uint32_t kMtB = kMtN;        // word offset of buffer B
constexpr uint32_t kMtPad = 2 * kMtN;  // the pad: a copy of A[0..15]
constexpr int kMtWin = 16;              // most words a locking lane prefetches (WIN)
__device__ __forceinline__ void mt_unpack(uint32_t r, int &idx, int &pg, int &cur) {
    idx = (int)(r & 0x3FFu);
    pg = (int)((r >> 10) & 0x3FFu);
    cur = (int)((r >> 20) & 1u);
}
__device__ __forceinline__ uint32_t mt_pack(int idx, int pg, int cur) {
    return (uint32_t)idx | ((uint32_t)pg << 10) | ((uint32_t)cur << 20);
}
// The preview (the piece the env's NEXT spawn takes, drawn one spawn ahead so
// that no step waits on a draw; see run_steps) in the upper bits of the same
// word: pv << 21 | ok << 24 | c << 25, c = the MT words its draw
// consumed (6 bits; a draw of > 62 words has p < 2^-62), so the reference's
// state -- the one before the preview was drawn -- is c words back
// (k_mt_sync).  ok = 0 (a host-written or synced state): the next spawn draws
// its piece first, then the preview.  Bit 31 is zero.  (Round 1 kept a
// 4-word draw-window cache per env flagged there; with the 64-word successor
// chunks the draw wave's window wait is off the critical chain, and the
// cache's 16 B per env and step bought nothing: removed, A/B +-0.)
constexpr uint32_t kMtLow = (1u << 21) - 1u;  // idx | pg | cur
constexpr uint32_t kPvOk = 1u << 24;
constexpr uint32_t kPvCMax = 63u;
__device__ __forceinline__ uint32_t mt_keep(uint32_t hi, uint32_t low) { return (hi & ~kMtLow) | low; }
__device__ __forceinline__ int pv_id(uint32_t r) { return (int)((r >> 21) & 7u); }
__device__ __forceinline__ bool pv_ok(uint32_t r) { return (r & kPvOk) != 0u; }
// words consumed between MT positions (idx0, cur0) and (idx1, cur1) (one
// generation switch at most: a draw consumes > 624 words with p < 2^-600)
__device__ __forceinline__ uint32_t mt_consumed(uint32_t before, uint32_t after) {
    const int i0 = (int)(before & 0x3FFu), i1 = (int)(after & 0x3FFu);
    const int c = ((before ^ after) >> 20) & 1u ? kMtN - i0 + i1 : i1 - i0;
    return (uint32_t)c < kPvCMax ? (uint32_t)c : kPvCMax;
}
__device__ __forceinline__ uint32_t pv_pack(uint32_t mt_after, int pv, uint32_t c) {
    return (mt_after & kMtLow) | ((uint32_t)pv << 21) | kPvOk | (c << 25);
}

// The wave's 64 MT states as one buffer resource.  Loads and stores of lanes
// (or operands) not wanted get an out-of-range offset (loads read 0), so each
// is issued on one path: no branch, and no merge of loaded and zeroed
// registers, which would make the compiler wait for the loads on the spot.
struct MtRes {
    __amdgpu_buffer_rsrc_t r;
    uint32_t lane_off;  // byte offset of this lane's buffer A
};
__device__ __forceinline__ MtRes mt_res(uint32_t *mt_wave, int lane) {
    MtRes m;
    m.r = buf_rsrc(mt_wave, (uint32_t)((kWave * kMtPitch + kMtPadBack) * 4));
    m.lane_off = (uint32_t)(lane * kMtPitch) * 4u;
    return m;
}
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4 mt_ld16(const MtRes &rs, bool on, uint32_t word) {
    return __builtin_amdgcn_raw_buffer_load_b128(rs.r, on ? rs.lane_off + 4u * word : kOff, 0, 0);
}

// The draw window: MT words cur[idx ..] of a locking lane, loaded
// right after the lock decision and consumed by the draw.  Reads past an
// env's state land in the next env's state or the allocation's back pad.
struct MtPre {
    uint32_t w[kMtWin];
};
// WIN = 8 for st_step (P(8 rejections) <= 2^-8: a dependent load for a few
// lanes per step, off the critical chain); 16 in rollouts.
template <int WIN>
__device__ __forceinline__ void mt_pre_load(const MtRes &rs, uint32_t mtst, bool want, MtPre &q) {
    int idx, pg, cur;
    mt_unpack(mtst, idx, pg, cur);
    const uint32_t cb = cur ? kMtB : 0u;
    u32x4 wv[WIN / 4];
#pragma unroll
    for (int i = 0; i < WIN / 4; ++i) wv[i] = mt_ld16(rs, want, cb + idx + 4 * i);
#pragma unroll
    for (int i = 0; i < WIN / 4; ++i)
        q.w[4 * i] = wv[i].x, q.w[4 * i + 1] = wv[i].y, q.w[4 * i + 2] = wv[i].z, q.w[4 * i + 3] = wv[i].w;
}
// Take all prefetched words at once (one vmcnt wait on a single path): words
// never read would stay "pending" for the compiler, and every later reuse of
// their registers would wait vmcnt(0), draining the step's early stores.
template <int WIN>
__device__ __forceinline__ void mt_win_consume(const MtPre &q) {
    asm volatile("" ::"v"(q.w[0]), "v"(q.w[1]), "v"(q.w[2]), "v"(q.w[3]), "v"(q.w[4]), "v"(q.w[5]),
                 "v"(q.w[6]), "v"(q.w[7]));
    if constexpr (WIN > 8)
        asm volatile("" ::"v"(q.w[8]), "v"(q.w[9]), "v"(q.w[10]), "v"(q.w[11]), "v"(q.w[12]),
                     "v"(q.w[13]), "v"(q.w[14]), "v"(q.w[15]));
}

// One 64-word chunk of one env's next generation per wave and step
// (wave-uniform).  mt_chunk_issue picks the lowest lane whose successor is
// incomplete and that has no preview straddling a generation switch (that
// preview's words sit in the buffer the successor is built into, and
// st_mt_sync may still give them back) and issues the operand loads:
// lane i computes next[k], k = p + i:
//   next[k] = X ^ mix(cur[k], cur[k + 1]),  X = cur[k + 397] (k < 227) | next[k - 227],
// which covers new[623] too (cur[624] = next[0], see the layout).  Every
// X = next[k - 227] lies >= 163 words below p: built by an earlier chunk.
struct MtChunk {
    uint32_t a0, a1, x;
    uint32_t base;  // byte offset of the chosen env's buffer A in the wave's MT resource
    int l;          // chosen lane (-1: none)
    int pg, cur;    // its progress and current buffer
};
// (cand, pg, cur: per lane; the chosen lane's progress and current buffer)
__device__ __forceinline__ void mt_chunk_issue_pc(const MtRes &rs, bool cand, int pg, int cur, int lane, MtChunk &c) {
    // branch-free: a load issued on one path only would be merged with a
    // zero at the join, and the merge waits for it on the spot (before B1)
    const uint64_t m = __ballot(cand);
    c.l = m ? (int)__builtin_ctzll(m) : -1;
    const int l = m ? c.l : 0;  // wave-uniform: v_readlane, not an LDS permute round trip
    c.pg = __builtin_amdgcn_readlane(pg, l);
    c.cur = __builtin_amdgcn_readlane(cur, l);
    c.base = (uint32_t)l * (uint32_t)kMtPitch * 4u;
    const int k = c.pg + lane;
    const bool on = m != 0 && k < kMtN;
    const uint32_t cb = c.cur ? kMtB : 0u, nb = c.cur ? 0u : kMtB;
    const uint32_t xo = k < 227 ? cb + (uint32_t)k + 397u : nb + (uint32_t)k - 227u;
    c.a0 = __builtin_amdgcn_raw_buffer_load_b32(rs.r, on ? c.base + 4u * (cb + (uint32_t)k) : kOff, 0, 0);
    c.a1 = __builtin_amdgcn_raw_buffer_load_b32(rs.r, on ? c.base + 4u * (cb + (uint32_t)k + 1u) : kOff, 0, 0);
    c.x = __builtin_amdgcn_raw_buffer_load_b32(rs.r, on ? c.base + 4u * xo : kOff, 0, 0);
}
__device__ __forceinline__ void mt_chunk_issue(const MtRes &rs, uint32_t mtw, bool real, int lane, MtChunk &c) {
    int idx, pg, cur;
    mt_unpack(mtw, idx, pg, cur);
    const int cc = (int)((mtw >> 25) & kPvCMax);
    mt_chunk_issue_pc(rs, real && pg < kMtN && !(pv_ok(mtw) && idx <= cc), pg, cur, lane, c);
}
// Compute and store the chunk (+ the pad copy of next[0..15] when next = A);
// returns the chosen env's new progress.  AUX: kNT in st_step; plain in
// rollouts, whose later steps read these words back (X operands, draws).
template <int AUX>
__device__ __forceinline__ int mt_chunk_store(const MtRes &rs, int lane, const MtChunk &c) {
    const int k = c.pg + lane;
    const bool on = c.l >= 0 && k < kMtN;
    const uint32_t v = c.x ^ mt_mix(c.a0, c.a1);
    const uint32_t nb = c.cur ? 0u : kMtB;
    __builtin_amdgcn_raw_buffer_store_b32(v, rs.r, on ? c.base + 4u * (nb + (uint32_t)k) : kOff, 0, AUX);
    __builtin_amdgcn_raw_buffer_store_b32(v, rs.r, on && c.cur && k < kMtWin ? c.base + 4u * (kMtPad + (uint32_t)k) : kOff,
                                          0, AUX);
    return c.pg + kWave < kMtN ? c.pg + kWave : kMtN;
}

// Finish the next generation of ONE env (words [pg, 624)), wave-cooperatively
// (out of line: inlined, its loop-invariant lane masks were hoisted into the
// rollout's prologue and pushed its step loop past the SGPR limit -- spills
// to VGPR lanes, reloaded every step; -5.5% packed rollout once out of line)
// (wave-uniform arguments): the chunked recurrence in LDS -- [0,227) reads old
// words | [227,454) reads [0,227) | [454,623) reads [227,396) | 623 reads 396
// and 0, each chunk only words that are old or finished.
__device__ __attribute__((noinline)) void mt_finish(uint32_t *g, uint32_t *S, int lane, int pg, int cur) {
    const uint32_t *src_new = g + (cur ? 0 : kMtB), *src_old = g + (cur ? kMtB : 0);
    uint32_t *dst = g + (cur ? 0 : kMtB);
    {
        uint32_t t[10];  // 624 = 9 * 64 + 48: issue all ten loads before any wait
#pragma unroll
        for (int q = 0; q < 10; ++q) {
            const int i = lane + kWave * q;
            t[q] = i < kMtN ? (i < pg ? src_new[i] : src_old[i]) : 0u;
        }
#pragma unroll
        for (int q = 0; q < 10; ++q) {
            const int i = lane + kWave * q;
            if (i < kMtN) S[i] = t[q];
        }
    }
    wave_sync();
    uint32_t v[4];
    auto chunk = [&](int lo, int hi, int xoff) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int k = lo + lane + kWave * q;
            if (k < hi && k >= pg) v[q] = S[k + xoff] ^ mt_mix(S[k], S[k + 1]);
        }
        wave_sync();
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int k = lo + lane + kWave * q;
            if (k < hi && k >= pg) S[k] = v[q];
        }
        wave_sync();
    };
    chunk(0, 227, 397);
    chunk(227, 454, -227);
    chunk(454, 623, -227);
    if (lane == 0 && pg <= 623) S[623] = S[396] ^ mt_mix(S[623], S[0]);
    wave_sync();
    for (int i = lane; i < kMtN; i += kWave)
        if (i >= pg) dst[i] = S[i];
    if (cur && lane < kMtWin) g[kMtPad + lane] = S[lane];
    __builtin_amdgcn_s_waitcnt(0);  // rare path: stores done before the wave reads them back
    wave_sync();
}

// The memory path of a draw: lanes still `pending` after their register
// words read 8 words at a time from the current generation, switching to the
// next one at index 624 (finishing it first where its chunks have not).
// Wave-uniform.  n, kb: randint's range and getrandbits width.
// FIN_ALL: a successor is finished from word 0 (the rollout whose output
// wave builds the chunks: their stores may still be in flight when it
// publishes the progress, so the progress is not trusted here; the words it
// rewrites are the same values)
template <bool FIN_ALL = false>
__device__ __forceinline__ void draw_slow(bool &pending, uint32_t &r, int &idx, int &pg, int &cur, uint32_t n, int kb,
                                          uint32_t *mt_wave, uint32_t *S, int lane) {
    if (__ballot(pending)) {
        const MtRes rs = mt_res(mt_wave, lane);
        do {
            // lanes at the end of their generation switch to the next one,
            // finishing it first where the chunks have not
            const bool sw = pending && idx >= kMtN;
            uint64_t fin = __ballot(sw && pg < kMtN);
            while (fin) {
                const int l = __builtin_ctzll(fin);
                fin &= fin - 1;
                mt_finish(mt_wave + (size_t)l * kMtPitch, S, lane, FIN_ALL ? 0 : __shfl(pg, l), __shfl(cur, l));
            }
            if (sw) {
                cur ^= 1;
                idx = 0;
                pg = 0;
            }
            const uint32_t cb = cur ? kMtB : 0u;
            const u32x4 w0 = mt_ld16(rs, pending, cb + idx), w1 = mt_ld16(rs, pending, cb + idx + 4);
            // both consumed here: the loop below may break before reading w1,
            // and a load still pending at the exit makes every later write of
            // its registers (reused by the caller) wait vmcnt(0)
            asm volatile("" ::"v"(w0.x), "v"(w0.y), "v"(w0.z), "v"(w0.w), "v"(w1.x), "v"(w1.y), "v"(w1.z),
                         "v"(w1.w));
            const uint32_t word[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (!__ballot(pending && idx < kMtN)) break;
                if (pending && idx < kMtN) {
                    const uint32_t y = mt_temper(word[j]) >> (32 - kb);
                    ++idx;
                    if (y < n) {
                        pending = false;
                        r = y;
                    }
                }
            }
        } while (__ballot(pending));
    }
}

// _choose_shape (tetris_env.py:183-191) + the count update of _new_piece
// (:199) for every lane with `need`: randint(1, sum(m)) = 1 + _randbelow(n)
// with rejection sampling on getrandbits(k) (Lib/random.py:239-249).  `mtst`
// is the lane's packed MT state (mt_pack).  Wave-uniform: every lane of the
// wave calls it.  `pre`: the window the caller loaded for lanes with
// `have_pre`.  The common case is branch-free: all 8 words tempered as
// independent chains, each lane takes its first accepted one; lanes the
// window does not settle (8 rejections, p <= 2^-8, or the generation's end)
// continue in the loop, switching generations at index 624.
// COUNT: also count the drawn shape in cnt (a spawn's _new_piece :199; not
// for a preview, which is counted when it spawns).
// pre_pg: the next generation's progress when `pre` was loaded (-1: now);
// its words past index 623 are usable only if that generation was complete.
// The count-dependent part of a draw (randint's range n = sum(m), its
// getrandbits width kb, and the prefix sums th[i] = m_0 + .. + m_i), split
// off so that st_step's draw wave computes it before the lock decision: the
// counts a spawn's preview draw sees are known at the start of the step
// (the counts then + the preview's own shape; clear() keeps shape_counts).
struct DrawPar {
    uint32_t n;
    int kb;
    int32_t th[6];
};
__device__ __forceinline__ DrawPar draw_par(const int32_t (&cnt)[7]) {
    int32_t maxc = cnt[0], sumc = cnt[0];
#pragma unroll
    for (int i = 1; i < 7; ++i) {
        maxc = cnt[i] > maxc ? cnt[i] : maxc;
        sumc += cnt[i];
    }
    DrawPar d;
    d.n = (uint32_t)(35 + 7 * maxc - sumc);
    d.kb = 32 - __builtin_clz(d.n);
    int32_t sum = 0;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        sum += 5 + maxc - cnt[i];
        d.th[i] = sum;
    }
    return d;
}
// The draw itself, for the lanes with `need` (see draw_shape): the window's
// words are tempered 4 at a time (acceptance >= 1/2, ~0.7 typically; a second
// group of 4 only in waves where a lane rejected 4 in a row), and the shape is
// the number of prefix sums <= r (the first i with r + 1 <= th[i], :186-191:
// independent compares, no serial chain).
template <int WIN>
__device__ __forceinline__ int draw_core(bool need, const DrawPar &dp, uint32_t &mtst, uint32_t *mt_wave,
                                         uint32_t *S, int lane, const MtPre &pre, bool have_pre, int pre_pg = -1) {
    const uint32_t n = dp.n;
    const int kb = dp.kb;
    int idx, pg, cur;
    mt_unpack(mtst, idx, pg, cur);
    bool pending = need;
    uint32_t r = 0;
    mt_win_consume<WIN>(pre);
    if (have_pre && pending) {
        // The prefetched words sit at positions idx.. of the current
        // generation and, past 623, of the next one (cur[624..639] is
        // next[0..15], see the layout) -- usable there once it is complete.
        const int lim = (pre_pg < 0 ? pg : pre_pg) == kMtN ? kMtN + WIN : kMtN;
        int pos = idx;  // words consumed, counted from the current generation's start
        // NW words w[0..NW) at positions p0.. (lanes continuing at p0 only)
        auto pass = [&](const uint32_t *w, int p0, auto nwc) {
            constexpr int NW = decltype(nwc)::value;
            int first = NW;
            uint32_t rr = 0;
#pragma unroll
            for (int j = NW - 1; j >= 0; --j) {
                const uint32_t y = mt_temper(w[j]) >> (32 - kb);
                const bool acc = y < n && p0 + j < lim;
                first = acc ? j : first;
                rr = acc ? y : rr;
            }
            if (first < NW) {
                pending = false;
                r = rr;
                pos = p0 + first + 1;
            } else {
                pos = p0 + NW < lim ? p0 + NW : lim;
            }
        };
        using I4 = std::integral_constant<int, 4>;
        using I8 = std::integral_constant<int, 8>;
        const int b = idx;
        if (pending) pass(pre.w, b, I4{});
        if (__ballot(pending && pos == b + 4)) {
            if (pending && pos == b + 4) pass(pre.w + 4, b + 4, I4{});
        }
        // 8 rejections in a row (p <= 2^-8 per draw, a few lanes per step):
        // the next 8 words are already here, no dependent load
        if constexpr (WIN > 8) {
            if (__ballot(pending && pos == b + 8)) {
                if (pending && pos == b + 8) pass(pre.w + 8, b + 8, I8{});
            }
        }
        if (pos > kMtN) {  // the draw ran into the (complete) next generation
            cur ^= 1;
            pos -= kMtN;
            pg = 0;
        }
        idx = pos;
    }
    draw_slow(pending, r, idx, pg, cur, n, kb, mt_wave, S, lane);
    if (need) mtst = mt_keep(mtst, mt_pack(idx, pg, cur));
    if (!need) return 0;
    int pick = 0;
#pragma unroll
    for (int i = 0; i < 6; ++i) pick += dp.th[i] <= (int32_t)r ? 1 : 0;
    return pick;
}
template <int WIN, bool COUNT = true>
__device__ __forceinline__ int draw_shape(bool need, int32_t (&cnt)[7], uint32_t &mtst,
                                          uint32_t *mt_wave, uint32_t *S, int lane,
                                          const MtPre &pre, bool have_pre, int pre_pg = -1) {
    const int pick = draw_core<WIN>(need, draw_par(cnt), mtst, mt_wave, S, lane, pre, have_pre, pre_pg);
    if constexpr (COUNT) {
#pragma unroll
        for (int i = 0; i < 7; ++i) cnt[i] += (need && i == pick);
    }
    return pick;
}

// The rollout's draw from a lane's register window (k_rollout, draw wave):
// `wv` holds the 16 MT words at the positions from where the window was
// loaded, of which the first `wlim` are valid (words past index 623 only if
// the next generation was complete then) and the first `o` already consumed
// (o may exceed 16: then none is left).  The 8 words at o.. are brought to the
// front by a 4-stage select network (the offset differs per lane), tempered
// as 8 independent chains, and each lane with `need` takes its first accepted
// getrandbits(k); lanes they do not settle continue from memory (draw_slow).
// Same rule as draw_shape (randint(1, sum(m)), tetris_env.py:183-191); `mta`
// (idx | pg | cur) and `o` advance past the words consumed.  Wave-uniform.
template <bool FIN_ALL>
__device__ __forceinline__ int draw_win(bool need, const int32_t (&cnt)[7], uint32_t &mta, const MtPre &wv, int &o,
                                        int wlim, uint32_t *mt_wave, uint32_t *S, int lane) {
    int32_t maxc = cnt[0], sumc = cnt[0];
#pragma unroll
    for (int i = 1; i < 7; ++i) {
        maxc = cnt[i] > maxc ? cnt[i] : maxc;
        sumc += cnt[i];
    }
    const uint32_t n = (uint32_t)(35 + 7 * maxc - sumc);
    const int kb = 32 - __builtin_clz(n);
    int idx, pg, cur;
    mt_unpack(mta, idx, pg, cur);
    const uint32_t before = mta & kMtLow;
    bool pending = need;
    uint32_t r = 0;
    {
        // m ? hi : lo bitwise, one v_bitop3 (truth table 0xE4 = (a & c) | (b & ~c));
        // a plain select here is recognised as a shifted array read and the
        // arrays go to scratch memory
        auto pick = [](uint32_t hi, uint32_t lo, uint32_t m) { return __builtin_amdgcn_bitop3_b32(hi, lo, m, 0xE4); };
        // the 8 words at o.. by a 3-stage network: o < 8 (a window is
        // reloaded after every draw, so o is the previous draw's few words;
        // o >= 8 takes the memory path)
        const int os = o & 7;
        const uint32_t m4 = 0u - (uint32_t)((os >> 2) & 1), m2 = 0u - (uint32_t)((os >> 1) & 1);
        const uint32_t m1 = 0u - (uint32_t)(os & 1);
        uint32_t b[11], c[9], w8[8];
#pragma unroll
        for (int j = 0; j < 11; ++j) b[j] = pick(wv.w[j + 4], wv.w[j], m4);
#pragma unroll
        for (int j = 0; j < 9; ++j) c[j] = pick(b[j + 2], b[j], m2);
#pragma unroll
        for (int j = 0; j < 8; ++j) w8[j] = pick(c[j + 1], c[j], m1);
        const int nv = o < 8 ? wlim - o : 0;  // valid words from o
        // words 0-3 tempered as independent chains (acceptance >= 1/2, ~0.7
        // typically: 4 rejections in a row are rare), 4-7 where a lane needs them
        // getrandbits(kb) = the top kb bits: with kb <= 18 on every lane
        // (n < 2^18: any counts the game itself produces) the tempering's
        // last step is skipped (mt_temper_hi18), and y >> (32 - kb) < n is
        // tested as y < n << (32 - kb), one shift for the accepted word
        const bool tail = __ballot(kb > 18) != 0;
        const uint32_t ns = n << (32 - kb);
        auto pass = [&](int j0) {
            int first = 4;
            uint32_t rr = 0;
            auto words = [&](auto tl) {
#pragma unroll
                for (int j = 3; j >= 0; --j) {
                    uint32_t y = mt_temper_hi18(w8[j0 + j]);
                    if constexpr (decltype(tl)::value) y ^= y >> 18;
                    const bool acc = y < ns && j0 + j < nv;
                    first = acc ? j : first;
                    rr = acc ? y : rr;
                }
            };
            if (tail) words(std::true_type{});
            else words(std::false_type{});
            rr >>= (32 - kb);
            if (pending) {
                int pos;
                if (first < 4) {
                    pending = false;
                    r = rr;
                    pos = idx + first + 1;
                } else {
                    const int left = nv - j0;  // valid words this pass had
                    pos = idx + (left < 0 ? 0 : (left < 4 ? left : 4));
                }
                if (pos > kMtN) {  // the draw ran into the (complete) next generation
                    cur ^= 1;
                    pos -= kMtN;
                    pg = 0;
                }
                idx = pos;
            }
        };
        pass(0);
        if (__ballot(pending && nv > 4)) pass(4);
    }
    draw_slow<FIN_ALL>(pending, r, idx, pg, cur, n, kb, mt_wave, S, lane);
    if (!need) return 0;
    mta = mt_pack(idx, pg, cur);
    o += (int)mt_consumed(before, mta);
    // the first i with r + 1 <= m_0 + .. + m_i (m_i = 5 + maxc - cnt[i],
    // :186-191) = the number of prefix sums below r + 1: independent
    // compares, no serial "found" chain
    int pick = 0, sum = 0;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        sum += 5 + maxc - cnt[i];
        pick += sum <= (int)r ? 1 : 0;
    }
    return pick;
}
// Valid words of a window loaded at MT position m (idx | pg | cur): up to
// index 623, or 639 when the next generation is complete (cur[624..639] is
// next[0..15], see the layout).
__device__ __forceinline__ int win_lim(uint32_t m) {
    const int idx = (int)(m & 0x3FFu), pg = (int)((m >> 10) & 0x3FFu);
    const int l = (pg == kMtN ? kMtN + kMtWin : kMtN) - idx;
    return l < kMtWin ? l : kMtWin;
}

// (x + 1) % lock_mod for l1 = x + 1 >= 1 (tetris_env.py:175): l1 <= lock_mod
// except after a host-written state (a lock field up to 2^15), which a
// division reduces -- only in a wave where some lane needs it (wave-uniform
// branch: a bounded cost once per host write, not a subtraction loop of up to
// 2^15 rounds; as a plain % the division ran, exec-masked, on every step)
__device__ __forceinline__ int lock_next(int l1, int lock_mod) {
    int r = l1 < lock_mod ? l1 : l1 - lock_mod;
    if (__ballot(r >= lock_mod)) r = r >= lock_mod ? r % lock_mod : r;
    return r;
}
__device__ __forceinline__ uint32_t pack_piece(int id, int rot, int ax, int ay, int lock) {
    return (uint32_t)id | ((uint32_t)rot << 3) | ((uint32_t)ax << 5) | ((uint32_t)ay << 11) |
           ((uint32_t)lock << 17);
}

// ---------------------------------------------------------------- step
// In-kernel phase stamps (diagnostic instantiation only; MI355X guide §7).
// st_step: the time at each stamp; st_rollout: the cycles from the previous
// stamp, summed over the launch's steps (per-phase totals, uint32).
#define ST_STAMP(i)                                                    \
    do {                                                               \
        if constexpr (STAMP) {                                         \
            __builtin_amdgcn_sched_barrier(0);                         \
            const uint64_t now_ = __builtin_amdgcn_s_memtime();        \
            if constexpr (KSTEPS == 1) {                               \
                tstamp[i] = now_;                                      \
            } else {                                                   \
                tacc[i] += (uint32_t)(now_ - tlast);                   \
                tlast = now_;                                          \
            }                                                          \
            __builtin_amdgcn_sched_barrier(0);                         \
        }                                                              \
    } while (0)

// LDS of the step kernels: one instance per workgroup, shared by its waves
// (the two-wave st_step hands data between them through it).  Plain words
// only (no vector-type members: a __shared__ object must be trivially
// constructible).
template <int WT, bool F32, int KSTEPS>
struct StepLds {
    static constexpr int kCols = (WT ? WT : kMaxW) + 2 * kPad;
    // board columns L[x + kPad][lane], all-ones walls at both ends
    uint32_t L[kCols * kWave] __attribute__((aligned(16)));
    // staged counter rows SS[r][lane] (r < 14: stats rows, 14: piece word)
    uint32_t SS[kHotQ * 4 * kWave] __attribute__((aligned(16)));
    uint32_t T2[2 * 28] __attribute__((aligned(8)));  // piece table {m, g}
    uint32_t S[kMtN];                                  // mt_finish scratch
    // st_step: per env board keep-mask, changed board columns
    uint32_t KM[KSTEPS == 1 ? kWave : 4] __attribute__((aligned(16)));
    uint32_t BD[KSTEPS == 1 ? kWave : 4] __attribute__((aligned(16)));
    // float32 obs writer (F32): per-lane obs words at stride W+1 (conflict-
    // free transposed reads) and the 16 float4 patterns of a 4-bit nibble
    uint32_t O[F32 ? kWave * (kMaxW + 1) : 1];
    float F4[F32 ? 64 : 4] __attribute__((aligned(16)));
    // st_step: the obs overlay plane, laid out like L
    uint32_t OV[KSTEPS == 1 ? kCols * kWave : 4] __attribute__((aligned(16)));
    // two-wave st_step hand-offs (see run_steps)
    uint32_t dump[kWave] __attribute__((aligned(16)));  // the logic wave's padding-row writes
    // (step-parity double buffers where a wave may write step t+1's value
    // before the other has read step t's)
    uint32_t lockm[2][2], drawm[2];
    uint32_t pick1[kWave];
    uint32_t mtw[2][KSTEPS == 1 ? 1 : kWave];  // rollouts: the draw wave's MT word after step t
    uint32_t f1, f2;  // = t + 1 once step t's draw mask / first picks are written
};

// Roles of run_steps.  st_step runs TWO waves per 64 envs: the logic wave
// (action, lock path, board / obs / counter outputs) and the draw wave (MT
// words, the next-generation block, the piece draw), so the draw no longer
// sits on the logic wave's chain.  That works because spawns take a piece
// drawn one spawn AHEAD (the "preview", kept in the MT state word): a spawn
// needs no draw result from the same step, and the draw wave's draw -- the
// next preview -- is only stored.  The reference's RNG sequence is unchanged
// (every spawn / reset still consumes the next draw, with the shape counts of
// that moment: the preview is drawn right after the previous spawn's count
// update, and counts change only at spawns); st_mt_sync rewinds the preview's
// words for the host.  k_rollout2 (KSTEPS == 0) runs the same two roles.
constexpr int kRoleL = 1;
constexpr int kRoleD = 2;

__device__ __forceinline__ void wg_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
// One-way LDS hand-off between the waves of a workgroup without a barrier
// (the writer must not wait for the reader).
//
// Ordering.  The flag is a workgroup-scope atomic; the writer's release fence
// and the reader's acquire fence are restricted to the LDS address space
// (the "local" memory-model-relaxation annotation of __builtin_amdgcn_fence):
// on gfx950 they lower to `s_waitcnt lgkmcnt(0)` only.  An unrestricted
// workgroup-scope fence would also wait `vmcnt(0)` -- every outstanding
// global load and store of the wave, e.g. the draw wave's MT window -- which
// is what a volatile access or an asm memory clobber here cost in round 1.
// With the fences, the data a writer stores before lds_flag_set happen-before
// the reader's accesses after lds_flag_wait in the C++ / HIP model, and no
// plain access races.
//
// Where a reader takes the flag AND the data it guards in one LDS round trip
// (the rollout's queue / action ring and consumption mask: the flag is read,
// the data are read right behind it, and the flag is checked after both
// return), the data are read as relaxed workgroup-scope atomics (lds_ld; the
// writers store them with lds_st), so there is no data race, and the order
// of the two reads rests on the hardware: the LLVM AMDGPU memory model
// (AMDGPUUsage, "Memory Model GFX942", which gfx950 follows) states that the
// LDS operations of a wavefront are executed in order, so no fence is needed
// between LDS accesses of one wavefront and `s_waitcnt lgkmcnt` only waits
// for their results.  The signal fences keep the compiler from reordering
// the two reads (they emit nothing).
// (LDS address space explicitly: through a generic pointer the accesses
// become flat_* instructions, which count in vmcnt and wait for it.)
typedef __attribute__((address_space(3))) uint32_t lds_u32;
__device__ __forceinline__ uint32_t lds_ld(const uint32_t *p) {
    return __hip_atomic_load((const lds_u32 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(uint32_t *p, uint32_t v) {
    __hip_atomic_store((lds_u32 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_flag_set(uint32_t *f, uint32_t v) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __hip_atomic_store((lds_u32 *)f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}
// The same without the release fence's lgkmcnt(0) wait: a wave's LDS
// operations execute in issue order, so a flag stored after the data lands
// after it (what lds_flag_get's readers rely on too).  The rollout's draw
// wave publishes its queue counter this way (round 5: -1.7%,
// profiles/r05/ab_rollout_queue_publish_nofence.txt).
__device__ __forceinline__ void lds_flag_set_inorder(uint32_t *f, uint32_t v) {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __hip_atomic_store((lds_u32 *)f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}
__device__ __forceinline__ void lds_flag_wait(uint32_t *f, uint32_t v) {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    while (__hip_atomic_load((lds_u32 *)f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != v)
        __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
// A progress counter read as a relaxed LDS atomic (no wait by itself).
__device__ __forceinline__ uint32_t lds_flag_get(uint32_t *f) {
    return __hip_atomic_load((lds_u32 *)f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// The same for a progress counter that the writer may have advanced past v.
__device__ __forceinline__ void lds_flag_wait_ge(uint32_t *f, uint32_t v) {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    while ((int32_t)(__hip_atomic_load((lds_u32 *)f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) - v) < 0)
        __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// ROLE = kRoleL / kRoleD: the logic or the draw wave of a workgroup.
// KSTEPS == 1: TetrisEngine.step once (st_step); KSTEPS == 0: p.k consecutive
// steps (k_rollout2, st_rollout above 4 workgroups per CU) with the board and
// counters kept in LDS between steps, actions read one step ahead, and
// per-step outputs at [t].  State is
// loaded once at the start and stored once at the end.
// SC0: the context has no scoring flags (the reference's defaults,
// tetris_env.py:126-137): those tests fold away at compile time (measured:
// the rollout loop otherwise holds each flag as a 64-bit lane mask at the
// SGPR limit, -5% packed rollout; st_step -1%).
// VEC (st_step_vec): the vector env's outputs -- with
// p.final_obs, an env reset in this step returns the reset obs (the empty
// board clear() returns, tetris_env.py:306-315, :405-411) and its terminal
// obs goes to final_obs; with p.info, every counter row after the step is
// written to info [ST_NSTAT][n] (the ep_* rows: the finished episode's where
// the env was reset, else 0).
template <int WT, int HT, bool F32, bool STAMP, int KSTEPS, bool SC0, int ROLE, bool VEC = false>
__device__ __forceinline__ void run_steps(const KParams &p, StepLds<WT, F32, KSTEPS> &sm) {
    static_assert(ROLE == kRoleL || ROLE == kRoleD, "run_steps: the logic or the draw wave");
    static_assert(!VEC || KSTEPS == 1, "VEC: st_step only");
    constexpr bool DO_L = ROLE == kRoleL;  // action, lock path, outputs
    constexpr bool DO_D = ROLE == kRoleD;  // MT words, next-generation block, draws
    [[maybe_unused]] uint64_t tstamp[12] = {};
    [[maybe_unused]] uint32_t tacc[12] = {};  // rollout stamp build: per-phase cycle totals
    [[maybe_unused]] uint64_t tlast = 0;
    [[maybe_unused]] uint64_t draw_kind = 0;  // stamp build: 1 = a lane twisted, 2 = a draw ran past 8 words
    constexpr bool S32 = HT != 0 && HT <= 25;  // see pc_bits
    const uint32_t kFlags = SC0 ? (p.flags & (ST_REWARD_STEP | ST_STEP_RESET)) : p.flags;

    // timing ablations (tools/ablate.sh) exist only in -DST_ABLATION=1 builds:
    // as runtime flags each costs two SGPRs of lane masks, and the rollout
    // loop is at the SGPR limit
#if defined(ST_ABLATION) && ST_ABLATION
    const uint32_t kAblate = p.ablate;
#else
    constexpr uint32_t kAblate = 0u;
#endif
    [[maybe_unused]] uint64_t rt0 = 0;
    if constexpr (STAMP) {
        rt0 = __builtin_amdgcn_s_memrealtime();
        tlast = __builtin_amdgcn_s_memtime();
    }
    ST_STAMP(0);
    if constexpr (ROLE == kRoleL && KSTEPS == 1) __builtin_amdgcn_s_setprio(kLogicPrio);
    uint32_t *const L = sm.L;
    uint32_t *const SS = sm.SS;
    const int W = WT ? WT : p.W;
    const int H = HT ? HT : p.H;
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t e0 = (int64_t)blockIdx.x * kWave;
    const int64_t e = e0 + lane;
    const int64_t sd = p.stride;
    const bool real = e < p.n;
    const uint32_t hmask = (1u << H) - 1u;
    const uint32_t floorb = ~hmask;

    // ---- loads: 16 B per lane (a wave's slice of one SoA row is 256 B) ----
    // Lane l covers row 4q + l/16, envs 4(l%16)..+3: one per-lane 32-bit offset
    // `loff` serves every 4-row group q (the group's base is wave-uniform), so
    // addresses are SGPR base + VGPR offset.  The board allocation is padded
    // to a multiple of 4 rows; rows >= W land in the right-wall LDS columns,
    // which are written after them.  Counter rows: 0..14 plus row 15 (unused).
    // Two waves: the logic wave loads the board and counter groups 0-1
    // (time .. count1), the draw wave groups 2-3 (count2 .. MT word, piece).
    const uint32_t loff = (uint32_t)(lane >> 4) * (uint32_t)sd + 4u * (uint32_t)(lane & 15);
    constexpr int NBQ = ((WT ? WT : kMaxW) + 3) / 4;  // board 4-row groups
    const uint32_t *bsrc = p.board + e0;
    // (ablation 1024: every wave's counter groups from the first workgroup's
    // lines -- the counter rows' HBM reads gone, timing only)
    const uint32_t *ssrc = reinterpret_cast<const uint32_t *>(p.stats) + ((kAblate & 1024u) ? 0 : e0);
    constexpr bool OVP = KSTEPS == 1;
    // st_step (not st_step_vec, whose info snapshot needs every counter of
    // every env): LATE COUNTERS.  The prologue's load burst carries only what
    // every env needs at the step start -- board, action, time, piece word,
    // MT word -- and the lock-only counter rows are read per locking lane
    // once the lock decision is known (logic: score .. deaths, issued before
    // B1, needed at the end of the lock path; draw: the shape counts, issued
    // with the MT window after B1)
    // (round 4, profiles/r04/ab_late_counters.txt: K = 2,000 4.642-4.643 ->
    // 4.605-4.635 us; reading the draw wave's shape counts late as well was
    // +6% -- its post-B1 chain, window + counts + draw parameters, became the
    // step's -- and was dropped)
    constexpr bool LCL = KSTEPS == 1 && !VEC;
    // staged counter groups (rows 4q .. 4q + 3): logic 0-1, draw 2-3; with
    // late rows only what the other role still reads early
    // LCL: the draw wave stages exactly the rows it reads, the shape counts
    // and the MT word (rows COUNT0 .. MT_INDEX: two 4-row groups from row 6,
    // a group's base row needs no alignment) -- round 4 staged rows 4..15,
    // 16 B per env more
    static_assert(ST_STAT_MT_INDEX == ST_STAT_COUNT0 + 7, "counts and MT word: 8 consecutive rows");
    auto mine_q = [&](int q) {
        if constexpr (LCL) return ROLE == kRoleD && (q == 1 || q == 2);
        return (ROLE == kRoleL) == (q < 2);
    };
    auto qbase = [&](int q) -> int {  // first stats row of staged group q
        if constexpr (LCL) return ST_STAT_COUNT0 + 4 * (q - 1);
        return 4 * q;
    };
    // Rows past the last real row (board padding, counter row 15) re-read the
    // last row -- the same cache line another lane fetches -- instead of
    // fetching padding; the loads stay unconditional (a load under a branch
    // costs a full vmcnt wait at the join).
    auto clamp_off = [&](int q, int nrows) -> uint32_t {
        const int r = 4 * q + (lane >> 4) < nrows ? (lane >> 4) : nrows - 1 - 4 * q;
        return (uint32_t)r * (uint32_t)sd + 4u * (uint32_t)(lane & 15);
    };
    uint4 bv[NBQ];
    if constexpr (DO_L) {
#pragma unroll
        for (int q = 0; q < NBQ; ++q)
            if (WT || 4 * q < W)
                bv[q] = *reinterpret_cast<const uint4 *>(bsrc + (size_t)(4 * q) * sd +
                                                         (4 * q + 4 <= W ? loff : clamp_off(q, W)));
    }
    // (four named registers, not an array: an array indexed in two unrolled
    // loops was once left in scratch memory)
    static_assert(kHotQ == 4, "four staged counter groups");
    uint4 sv0 = make_uint4(0u, 0u, 0u, 0u), sv1 = sv0, sv2 = sv0, sv3 = sv0;
    auto ldq = [&](int q) -> uint4 {
        return *reinterpret_cast<const uint4 *>(ssrc + (size_t)qbase(q) * sd +
                                                (qbase(q) + 4 <= kHotRows ? loff : clamp_off(q, kHotRows)));
    };
    if (mine_q(0)) sv0 = ldq(0);
    // (ablation 262144: st_step's draw wave does not load shape counts T J L Z -- timing only)
    if (mine_q(1) && !(LCL && (kAblate & 262144u))) sv1 = ldq(1);
    if (mine_q(2)) sv2 = ldq(2);
    if (mine_q(3)) sv3 = ldq(3);
    const int K = KSTEPS ? KSTEPS : p.k;
    // two-wave st_step: the logic wave also builds the next-generation block
    // (the draw wave's chain is the longer one).  (Measured and dropped: the
    // draw wave running the action phase itself instead of waiting at B1 --
    // the two concurrent action phases slowed the logic wave's by ~50%.)
    constexpr bool STEP2 = KSTEPS == 1;
    constexpr bool ACT = DO_L;
    // unconditional (clamped) so it is issued with the others; masked at use
    uint32_t act_next = 0;
    if constexpr (ACT) act_next = p.actions[real ? e : p.n - 1];
    // st_gate_actions (VEC instantiations, which every gated launch uses):
    // the gate word, loaded with the prologue's burst (an empty range reads 0
    // when the launch is not gated), tested after B0 -- before any global
    // store of either wave
    [[maybe_unused]] uint32_t gate_v = 0;
    if constexpr (VEC) gate_v = __builtin_amdgcn_raw_buffer_load_b32(buf_rsrc(p.gate, 4u), 0u, 0, 0);
    // two-wave st_step: the logic wave also fetches its piece word and clock
    // per env (4 B/lane from lines the state loads fetch anyway), so the
    // action phase starts from registers instead of an LDS read after B0
    // (A/B: -0.2%)
    constexpr bool DL = KSTEPS == 1 && ROLE == kRoleL;
    [[maybe_unused]] uint32_t pw_d = 0, tm_d = 0;
    if constexpr (DL) {
        pw_d = p.piece[e];
        tm_d = reinterpret_cast<const uint32_t *>(p.stats)[(int64_t)ST_STAT_TIME * sd + e];
    }
    // The piece table, lane i = entry i, from immediates (under the load
    // latency; no memory access: a __constant__ load gets sunk by the
    // compiler past the state loads' completion -- one more serialized round
    // trip).  Two waves: the draw wave builds it (and the walls, and the f32
    // nibble table).
    constexpr bool BUILD = DO_D;
    uint32_t tab_m = 0, tab_g = 0;
    if constexpr (BUILD) {
        // one v_writelane per entry (the constant in an SGPR: SALU): 56 VALU
        // instead of a compare + two selects per entry (~140 VALU), on the
        // draw wave's path to B0
#pragma unroll
        for (int i = 0; i < 28; ++i) {
            asm("v_writelane_b32 %0, %1, %2" : "+v"(tab_m) : "s"(kTab.m[i]), "i"(i));
            asm("v_writelane_b32 %0, %1, %2" : "+v"(tab_g) : "s"(kTab.g[i]), "i"(i));
        }
    }
    const int lrow = lane >> 4, lcc = 4 * (lane & 15);  // this lane's row-in-group, env slot
    if constexpr (DO_L) {
#pragma unroll
        for (int q = 0; q < NBQ; ++q) {
            // rows >= W (allocation padding) land in the right-wall columns:
            // one wave writes them first and the walls over them; the logic
            // wave of two sends them to a dump slot (the draw wave writes the
            // walls) -- an address select, not a branch: a store under a
            // branch gets its load sunk into the branch, one more round trip
            if (WT || 4 * q < W) {
                uint4 v = bv[q];
                v.x |= floorb;
                v.y |= floorb;
                v.z |= floorb;
                v.w |= floorb;
                uint32_t *dst = &L[(4 * q + lrow + kPad) * kWave + lcc];
                if constexpr (ROLE == kRoleL) dst = 4 * q + lrow < W ? dst : &sm.dump[lcc];
                *reinterpret_cast<uint4 *>(dst) = v;
            }
        }
    }
    if constexpr (BUILD) {
#pragma unroll
        for (int x = 0; x < kPad; ++x) {
            L[x * kWave + lane] = ~0u;
            L[(W + kPad + x) * kWave + lane] = ~0u;
        }
        if (lane < 28) {
            sm.T2[2 * lane] = tab_m;
            sm.T2[2 * lane + 1] = tab_g;
        }
        if constexpr (F32) {
            if (lane < 16) {
                sm.F4[4 * lane] = (float)(lane & 1);
                sm.F4[4 * lane + 1] = (float)((lane >> 1) & 1);
                sm.F4[4 * lane + 2] = (float)((lane >> 2) & 1);
                sm.F4[4 * lane + 3] = (float)((lane >> 3) & 1);
            }
        }
    }
    auto stq = [&](int q, const uint4 &v) { *reinterpret_cast<uint4 *>(&SS[(qbase(q) + lrow) * kWave + lcc]) = v; };
    if (mine_q(0)) stq(0, sv0);
    if (mine_q(1)) stq(1, sv1);
    if (mine_q(2)) stq(2, sv2);
    if (mine_q(3)) stq(3, sv3);
    if constexpr (OVP && DO_L) {
#pragma unroll
        for (int q = 0; q < NBQ; ++q)
            if ((WT || 4 * q < W) && 4 * q + lrow < W)
                *reinterpret_cast<uint4 *>(&sm.OV[(4 * q + lrow + kPad) * kWave + lcc]) = make_uint4(0u, 0u, 0u, 0u);
    }
    if (ROLE == kRoleL && lane == 0) sm.f1 = 0u;
    if (ROLE == kRoleD && lane == 0) sm.f2 = 0u;
    wg_barrier();  // B0: the staged state is complete
    if constexpr (VEC) {
        // a gate that saw an action outside 0..6: no env steps (both waves
        // leave here, before B1 and before any global store)
        if (p.gate && __builtin_amdgcn_readfirstlane(gate_v) == p.gate_epoch) return;
    }
    auto ss = [&](int r) -> uint32_t & { return SS[r * kWave + lane]; };
    auto tab = [&](int i) -> uint2 { return *reinterpret_cast<const uint2 *>(&sm.T2[2 * i]); };
    // an action outside value_action_map in any step of this launch (the
    // reference's KeyError, tetris_env.py:245; the step treats it as idle)
    [[maybe_unused]] bool bad_act = false;
    for (int t = 0; t < K; ++t) {
    // ---------------- logic: action, gravity, lock decision ----------------
    uint32_t act = 6u;
    if constexpr (ACT) {
        act = real ? act_next : 6u;
        bad_act |= act > 6u;
        if (KSTEPS != 1 && t + 1 < K) act_next = p.actions[(int64_t)(t + 1) * p.n + (real ? e : p.n - 1)];
    }
    uint32_t *const obs_t = p.obs ? p.obs + (int64_t)t * W * p.n : nullptr;
    const uint32_t pw = DL ? pw_d : ss(kPieceRow);
    int32_t time = (int32_t)(DL ? tm_d : ss(ST_STAT_TIME));
    const int id = (int)(pw & 7u);
    int rot = (int)((pw >> 3) & 3u);
    int ax = (int)((pw >> 5) & 63u);
    int ay = (int)((pw >> 11) & 63u);
    int lock = (int)(pw >> 17);
    // MT word at the start of the step (the logic wave uses only the preview
    // bits; in a two-wave step the draw wave replaces the row after B1, and in
    // a two-wave rollout it hands step t-1's word over in mtw: read after B1)
    uint32_t mt0 = ss(ST_STAT_MT_INDEX);
    if constexpr (STAMP && KSTEPS == 1) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    ST_STAMP(1);

    uint2 desc = make_uint2(0u, 0u);
    bool locknow = false;
    int32_t rew = 0;
    // st_step's obs overlay of a spawn: its preview's descriptor, read in the
    // action phase's LDS round trip (not on the store phase's chain)
    [[maybe_unused]] uint2 pd_pv = make_uint2(0u, 0u);
    if constexpr (ACT) {
        // ---- action (tetris_env.py:245; value_action_map :152-160) + drop ----
        // Current and candidate descriptors and their columns are read in one
        // LDS round trip each; the collision and drop tests are then pure VALU.
        const bool tries = act == 0u || act == 1u || act == 4u || act == 5u;
        const int cx = ax + (act == 0u ? -1 : (act == 1u ? 1 : 0));
        const int cr = (rot + (act == 4u ? 1 : 0) + (act == 5u ? 3 : 0)) & 3;  // (selects: the ternary chain became an exec-mask branch)
        desc = tab(id * 4 + rot);
        const uint2 cdesc = tab(id * 4 + cr);
        if constexpr (OVP && DO_L) pd_pv = tab(pv_id(mt0) * 4);
        uint32_t cur[4], cand[4];
        read_cols(L, lane, desc.y, ax, cur);
        read_cols(L, lane, cdesc.y, cx, cand);
        // branch-free: select the accepted position's descriptor and columns, then
        // one drop test (both arms would otherwise run in a divergent wave)
        const bool ok = tries && !collides_v<S32>(cdesc.x, ay, cand);
        ax = ok ? cx : ax;
        rot = ok ? cr : rot;
        desc.x = ok ? cdesc.x : desc.x;
        desc.y = ok ? cdesc.y : desc.y;
#pragma unroll
        for (int j = 0; j < 4; ++j) cur[j] = ok ? cand[j] : cur[j];
        int d = drop_v(desc.y, ay, cur);
        if (act == 2u) {                 // hard_drop :54-59
            ay += d;
            d = 0;
        } else if (act == 3u && d > 0) { // soft_drop :49-51
            ay += 1;
            d -= 1;
        }
        // ---- gravity + lock delay (tetris_env.py:247-262) ----
        if (d > 0) {
            ay += 1;
            d -= 1;
            if (kFlags & ST_STEP_RESET) lock = 0;
        }
        time += 1;
        rew = (kFlags & ST_REWARD_STEP) ? 1 : 0;
        if (d == 0) {
            const int l1 = lock + 1;  // (x + 1) % lock_mod; x < lock_mod unless set_state said otherwise
            lock = lock_next(l1, p.lock_mod);
            locknow = lock == 0 && !(kAblate & 1u);
        }
    }
    ST_STAMP(2);
    // LC: the logic wave's lock-path counters, per locking lane (an
    // out-of-range offset elsewhere: no traffic, 0)
    [[maybe_unused]] uint32_t lcv[5] = {};
    if constexpr (LCL && DO_L) {
        const auto rs = buf_rsrc(p.stats, (uint32_t)kHotRows * (uint32_t)sd * 4u);
        // (ablation 8192: from the first workgroup's lines -- their HBM reads gone, timing only)
        const uint32_t eo = (kAblate & 8192u) ? (uint32_t)lane * 4u : (uint32_t)e * 4u;
#pragma unroll
        for (int j = 0; j < 5; ++j)  // (ablation 2097152: not loaded, timing only)
            lcv[j] = __builtin_amdgcn_raw_buffer_load_b32(
                rs, locknow && !(kAblate & 2097152u) ? eo + (uint32_t)(ST_STAT_SCORE + j) * (uint32_t)sd * 4u : kOff,
                0, 0);
    }
    // the draw wave's next-generation chunk of this step: operands issued
    // before B1, so they arrive while it waits for the lock decision
    [[maybe_unused]] MtChunk chunk;
    [[maybe_unused]] MtRes mrs;
    // ... and the count-dependent part of the preview draw (in st_step while
    // the draw wave waits for the lock decision): a lane that draws spawns its
    // preview first, so its draw sees the counts now + that shape (lanes
    // without a valid preview redo this after their first draw, below)
    [[maybe_unused]] int32_t cnt[7];
    [[maybe_unused]] DrawPar dpar;
    [[maybe_unused]] int32_t csid = 0;  // the spawned shape's count after the spawn
    if constexpr (DO_D) {
        mrs = mt_res(p.mt + e0 * kMtPitch, lane);
        mt_chunk_issue(mrs, mt0, real && !(kAblate & (2u | 1048576u)), lane, chunk);  // (1048576: no chunks, timing only)
        const int s0 = pv_id(mt0);
#pragma unroll
        for (int i = 0; i < 7; ++i) cnt[i] = (int32_t)ss(ST_STAT_COUNT0 + i) + (i == s0);  // _new_piece :199
        csid = cnt[0];
#pragma unroll
        for (int i = 1; i < 7; ++i) csid = s0 == i ? cnt[i] : csid;
        dpar = draw_par(cnt);
    }
    if constexpr (DO_L) {
        const uint64_t m = __ballot(locknow);
        if (lane == 0) {
            sm.lockm[t & 1][0] = (uint32_t)m;
            sm.lockm[t & 1][1] = (uint32_t)(m >> 32);
        }
    }
    wg_barrier();  // B1: the draw wave learns which lanes lock
    if constexpr (DO_D || KSTEPS != 1) ST_STAMP(10);
    if constexpr (DO_D) __builtin_amdgcn_s_setprio(kDrawPrio);
    if constexpr (DO_D) {
        const uint32_t w = lane < 32 ? sm.lockm[t & 1][0] : sm.lockm[t & 1][1];
        locknow = (w >> (lane & 31)) & 1u;
    }
    if constexpr (DO_L && KSTEPS != 1) {
        if (t > 0) mt0 = sm.mtw[(t - 1) & 1][lane];
    }

    // ---------------- draw: MT window, issued now ----------------
    // Every locking lane draws (its next preview, or -- without a valid
    // preview -- its piece first); the window is consumed after the lock path
    // in one wave, or right away by the draw wave.
    uint32_t mtst = mt0;  // packed (mt_pack + preview bits)
    const bool want_pre = locknow && !(kAblate & 2u);
    constexpr int kWin = STEP2 ? 8 : 16;
    MtPre pre;
    // (ablation 524288: the window's words read as zeros, no traffic -- timing only)
    if constexpr (DO_D) mt_pre_load<kWin>(mrs, mtst, want_pre && !(kAblate & 524288u), pre);

    // st_step's wide packed obs path (16-B stores of 4-env groups, below)
    [[maybe_unused]] const bool wide_obs1 = OVP && (p.n & 3) == 0 && e0 + kWave <= p.n &&
                                            (reinterpret_cast<uintptr_t>(p.obs) & 15u) == 0 &&
                                            (!VEC || (reinterpret_cast<uintptr_t>(p.final_obs) & 15u) == 0);

    // ---------------- logic: lock path (tetris_env.py:263-299) ----------------
    bool died = false, spawn = false;
    int32_t score = 0, lines = 0, holes = 0, height = 0, deaths = 0;
    int32_t o_score = 0, o_lines = 0, o_holes = 0, o_height = 0, o_deaths = 0;  // (dirty tests)
    [[maybe_unused]] bool hset = false;  // LC: height set by the lock path
    uint32_t bdirty = 0;  // st_step: board columns this step changes (stores skip the rest)
    if (DO_L && locknow) {
        // (LC: score / lines / deaths count from 0 here -- deltas, added to
        // the late-loaded values where they are stored, long after the lock
        // path; the old holes / height are read only by the scoring flags
        // that need them)
        if constexpr (!LCL) {
            score = o_score = (int32_t)ss(ST_STAT_SCORE);
            lines = o_lines = (int32_t)ss(ST_STAT_LINES);
            holes = o_holes = (int32_t)ss(ST_STAT_HOLES);
            height = o_height = (int32_t)ss(ST_STAT_PIECE_HEIGHT);
            deaths = o_deaths = (int32_t)ss(ST_STAT_DEATHS);
        }
        paint<S32>(L, lane, desc.x, desc.y, ax, ay, hmask);
        // Column words carry the floor bits, so the topmost cell of column v
        // is ctz(v) (H when empty) and its holes are H - ctz(v) - popc(v & hmask):
        // summed, holes = W*H - sum ctz(v) - (sum popc(v) - W*(32-H)).
        uint32_t andv = ~0u, orv = 0, sctz = 0, spop = 0;
        // (compile-time width: all W column reads issued before any is used,
        // one LDS round trip -- left to itself the scheduler reused the first
        // reads' registers as accumulators and issued the last pair after
        // waiting for the others; the clear path reuses the words)
        [[maybe_unused]] uint32_t cw[WT ? WT : 1];
        if constexpr (WT != 0) {
#pragma unroll
            for (int x = 0; x < WT; ++x) cw[x] = lcol(L, x, lane);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int x = 0; x < WT; ++x) {
                const uint32_t v = cw[x];
                andv &= v;
                orv |= v;
                sctz += __builtin_ctz(v);
                spop += __builtin_popcount(v);
            }
        } else {
#pragma unroll 8
            for (int x = 0; x < W; ++x) {
                const uint32_t v = lcol(L, x, lane);
                andv &= v;
                orv |= v;
                sctz += __builtin_ctz(v);
                spop += __builtin_popcount(v);
            }
        }
        andv &= hmask;
        if constexpr (KSTEPS == 1) {
#pragma unroll
            for (int j = 0; j < 4; ++j) bdirty |= 1u << (ax + pc_dx(desc.y, j));
            if (andv) bdirty = ~0u;
        }
        int32_t ncl = 0;
        if (andv) {  // full rows: compact, recount
            ncl = __builtin_popcount(andv);
            orv = 0;
            sctz = spop = 0;
            if constexpr (WT != 0) {
                // the columns in registers, one full row per round for all of
                // them (compact()'s steps in the same order): the rounds are
                // the wave's largest clear count, not one loop per column
                uint32_t c[WT];
#pragma unroll
                for (int x = 0; x < WT; ++x) c[x] = cw[x] & hmask;
                uint32_t full = andv;
                while (full) {
                    const int r = __builtin_ctz(full);
                    full &= full - 1u;
                    const uint32_t above = (1u << r) - 1u;
                    const uint32_t keep = ~(above | (1u << r));
#pragma unroll
                    for (int x = 0; x < WT; ++x) c[x] = (c[x] & keep) | ((c[x] & above) << 1);
                }
#pragma unroll
                for (int x = 0; x < WT; ++x) {
                    const uint32_t v = c[x] | floorb;
                    lcol(L, x, lane) = v;
                    orv |= v;
                    sctz += __builtin_ctz(v);
                    spop += __builtin_popcount(v);
                }
            } else {
#pragma unroll 8
                for (int x = 0; x < W; ++x) {
                    const uint32_t v = compact(lcol(L, x, lane) & hmask, andv) | floorb;
                    lcol(L, x, lane) = v;
                    orv |= v;
                    sctz += __builtin_ctz(v);
                    spop += __builtin_popcount(v);
                }
            }
            lines += ncl;
        }
        orv &= hmask;
        const int32_t nh = W * H - (int32_t)sctz - ((int32_t)spop - W * (32 - H));
        if (kFlags & ST_ADVANCED_CLEARS) {  // :266-269, 2.5 * [0,40,100,300,1200]
            // [0, 40, 100, 300, 1200][ncl] as 12-bit fields of one constant
            // (ncl > 4 only from a crafted set_state board: 0, as before)
            constexpr uint64_t kClr = (40ull << 12) | (100ull << 24) | (300ull << 36) | (1200ull << 48);
            const int32_t sc = ncl <= 4 ? (int32_t)((kClr >> (12 * ncl)) & 0xFFFu) : 0;
            rew += (sc * 5) / 2;
            score += sc;
        } else if (kFlags & ST_HIGH_SCORING) {  // :270-272
            rew += 1000 * ncl;
            score += ncl;
        } else {  // :273-275
            rew += 100 * ncl;
            score += ncl;
        }
        if (orv & 1u) {  // death :277-281
            holes = nh;
            deaths += 1;
            died = true;
            rew = -100;
        } else {  // :283-299
            const int32_t old_holes = LCL ? 0 : holes;
            holes = nh;
            const int32_t hgt = __builtin_popcount(orv);  // sum(np.any(board, axis=0))
            if (kFlags & ST_PENALISE_HEIGHT) {
                rew -= hgt;
            } else if (kFlags & ST_PENALISE_HEIGHT_INCREASE) {
                const int32_t oh = LCL ? (int32_t)lcv[3] : height;
                if (hgt > oh) rew -= 10 * (hgt - oh);
                height = hgt;
                hset = true;
            }
            if (kFlags & ST_PENALISE_HOLES) rew -= 5 * holes;
            else if (kFlags & ST_PENALISE_HOLES_INCREASE) rew -= 5 * (holes - (LCL ? (int32_t)lcv[2] : old_holes));
            spawn = true;
        }
    }
    ST_STAMP(3);

    const bool reset_now = died && p.autoreset == ST_AUTORESET_SAME_STEP;
    // a lock consumes the preview (spawn, or the same-step reset's new piece);
    // a death without auto-reset does not (the next st_reset takes it)
    bool draw = spawn || reset_now;
    if (DO_L && p.autoreset != ST_AUTORESET_SAME_STEP) {
        const uint64_t m = __ballot(draw);
        if (lane == 0) {
            sm.drawm[0] = (uint32_t)m;
            sm.drawm[1] = (uint32_t)(m >> 32);
            lds_flag_set(&sm.f1, (uint32_t)t + 1u);
        }
    }
    uint2 odesc = desc;
    int oax = ax, oay = ay;
    if constexpr (DO_L) {
        // reward / done never depend on the piece drawn below.  Buffer stores
        // (buf_rsrc): vmcnt counts loads and stores in issue order, and a store
        // skipped on some path would make a later load's wait vmcnt(0).
        const auto rr = buf_rsrc(p.reward ? p.reward + (int64_t)t * p.n : nullptr, (uint32_t)p.n * 4u);
        const auto rd = buf_rsrc(p.done ? p.done + (int64_t)t * p.n : nullptr, (uint32_t)p.n);
        __builtin_amdgcn_raw_buffer_store_b32(rew, rr, real ? (uint32_t)e * 4u : kOff, 0, kRD);
        __builtin_amdgcn_raw_buffer_store_b8((char)(died ? 1 : 0), rd, real ? (uint32_t)e : kOff, 0, kRD);
        if constexpr (KSTEPS == 1) ST_STAMP(10);  // (logic wave, round 6: reward / done stores issued)
    }
    if constexpr (DO_L && KSTEPS == 1) {
        // The post-step board never depends on the spawned piece either (a
        // spawn only overlays row 0, which is empty after a non-fatal lock,
        // :277), so st_step stores it here: non-locking lanes and spawns: L; a
        // death without auto-reset: L minus the locked piece (R8:
        // _set_piece(False), :303); a same-step reset: the empty board.  The
        // obs overlay of every non-spawning lane is then painted (a death's
        // terminal obs = L with its piece, :301).
        // Only rows (board columns x) that one of the lane's 4 envs changed are
        // written (buffer stores, see buf_rsrc).
        if (died && !reset_now) erase<S32>(L, lane, desc.x, desc.y, ax, ay, hmask);
        if (died) bdirty = ~0u;
        if constexpr (OVP) {
            // the overlay of every lane into its own plane: the current piece,
            // or for a spawn its new piece at the spawn position -- the
            // preview, known since the step started, or (rare: no preview)
            // the draw wave's first draw, waited for here
            // (the preview's descriptor was read with the action's)
            uint2 pd = pd_pv;
            const bool need1 = draw && !pv_ok(mt0);
            if (__ballot(need1)) {
                lds_flag_wait(&sm.f2, (uint32_t)t + 1u);
                if (need1) pd = tab((int)sm.pick1[lane] * 4);
            }
            const uint32_t om = spawn ? pd.x : desc.x, og = spawn ? pd.y : desc.y;
            const int ox = spawn ? W / 2 : ax, oy = spawn ? 0 : ay;
#pragma unroll
            for (int j = 0; j < 4; ++j)  // (ablation 4194304: skipped, timing only)
                if (!(kAblate & 4194304u)) sm.OV[(ox + pc_dx(og, j) + kPad) * kWave + lane] = pc_bits<S32>(om, j, oy) & hmask;
        }
        uint4 km, bd4;
        uint4 bw[NBQ], ow[NBQ];
        if (kAblate & 4194304u) {
            // (ablation 4194304: the store phase's LDS transposition skipped --
            // no keep / dirty mask or overlay writes, no row reads; the stores
            // take register garbage; timing only)
            km = make_uint4(hmask, hmask, hmask, hmask);
            bd4 = make_uint4(bdirty, bdirty, bdirty, bdirty);
#pragma unroll
            for (int q = 0; q < NBQ; ++q) {
                bw[q] = make_uint4(bdirty, (uint32_t)ax, (uint32_t)ay, (uint32_t)lane);
                ow[q] = make_uint4(desc.x, desc.y, (uint32_t)rew, (uint32_t)q);
            }
        } else {
        sm.KM[lane] = reset_now ? 0u : hmask;
        sm.BD[lane] = bdirty;
        wave_sync();
        km = *reinterpret_cast<const uint4 *>(&sm.KM[lcc]);
        bd4 = *reinterpret_cast<const uint4 *>(&sm.BD[lcc]);
#pragma unroll
        for (int q = 0; q < NBQ; ++q) {
            if (WT || 4 * q < W) {
                bw[q] = *reinterpret_cast<const uint4 *>(&L[(4 * q + lrow + kPad) * kWave + lcc]);
                if constexpr (OVP) ow[q] = *reinterpret_cast<const uint4 *>(&sm.OV[(4 * q + lrow + kPad) * kWave + lcc]);
            }
        }
        }
        // every read (keep / dirty masks, board and overlay rows) issued before
        // anything uses one: one LDS round trip
        // (the masks pass through an empty volatile asm placed after the row
        // reads: their first use cannot float above those reads -- it did,
        // splitting the batch in two round trips)
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("" : "+v"(km.x), "+v"(km.y), "+v"(km.z), "+v"(km.w), "+v"(bd4.x), "+v"(bd4.y), "+v"(bd4.z),
                     "+v"(bd4.w));
        if constexpr (STAMP) {  // (round 6: the row reads arrived, before the first store)
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            ST_STAMP(11);
        }
        const uint32_t bdl = (bd4.x | bd4.y | bd4.z | bd4.w) >> lrow;
        // the board array as one resource: byte offsets < W * stride * 4 <= 2^31
        const auto rb = buf_rsrc(p.board, (uint32_t)W * (uint32_t)sd * 4u);
        const uint32_t boff = ((uint32_t)e0 * 4u + loff * 4u);
        // obs rows board | overlay (a reset env's terminal board included):
        // no branch around the stores (a store on one path only made the
        // compiler wait for every LDS read at the join) -- a null range
        // drops them when the obs go the per-lane way below (or nowhere),
        // and rows past W lie past the range
        [[maybe_unused]] const auto ro = buf_rsrc(wide_obs1 ? p.obs : nullptr, (uint32_t)W * (uint32_t)p.n * 4u);
        [[maybe_unused]] const auto rf = buf_rsrc(VEC && wide_obs1 ? p.final_obs : nullptr,
                                                  (uint32_t)W * (uint32_t)p.n * 4u);
#pragma unroll
        for (int q = 0; q < NBQ; ++q) {
            if (WT || 4 * q < W) {
                uint4 v = bw[q];
                if constexpr (OVP) {
                    const uint4 o = ow[q];
                    const uint4 ob = make_uint4((v.x | o.x) & hmask, (v.y | o.y) & hmask, (v.z | o.z) & hmask,
                                                (v.w | o.w) & hmask);
                    const uint32_t ooff =
                        ((uint32_t)e0 + (uint32_t)(4 * q + lrow) * (uint32_t)p.n + (uint32_t)lcc) * 4u;
                    if constexpr (VEC) {
                        // reset envs (km = 0): the reset obs here, the
                        // terminal one to final_obs (groups with a reset)
                        const bool fin = !(km.x && km.y && km.z && km.w);
                        buf_store16<kNT>(rf, fin ? ooff : kOff, ob);
                        const uint4 keep = p.final_obs ? km : make_uint4(~0u, ~0u, ~0u, ~0u);
                        buf_store16<kNT>(ro, ooff, make_uint4(ob.x & keep.x, ob.y & keep.y, ob.z & keep.z, ob.w & keep.w));
                    } else {
                        buf_store16<kNT>(ro, ooff, ob);
                    }
                }
                v.x &= km.x;
                v.y &= km.y;
                v.z &= km.z;
                v.w &= km.w;
                // row 4q + lrow; padding rows (>= W) are never dirty
                const bool dirty = ((bdl >> (4 * q)) & 1u) && 4 * q + lrow < W && !(kAblate & 4096u);
                buf_store16<kST>(rb, dirty ? boff + (uint32_t)(4 * q) * (uint32_t)sd * 4u : kOff, v);
            }
        }
        // (below: the ragged / unaligned obs path and the float32 writer read
        // the planes per env; nothing is painted into L)
    }

    ST_STAMP(8);  // (stamp 8: between the early stores and the draw)
    // ---------------- draw (tetris_env.py:183-199, :299 _new_piece, :306-315 clear) ----------------
    // spawn id: the preview; lanes without one draw their piece first
    int sid = pv_id(mt0);
    if constexpr (DO_D) {
        // speculative in the draw wave (it does not know yet which locking
        // lanes die without auto-reset): committed below only where `draw`
        const bool dr_spec = locknow;
        if constexpr (STAMP) {  // diagnostic split of the draw: MT-word wait | compute
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            ST_STAMP(9);
        }
        [[maybe_unused]] const uint32_t mt_before = mtst;
        uint32_t mt_new = mtst;
        if (!(kAblate & 2u)) {
            mt_win_consume<kWin>(pre);
            const bool need1 = dr_spec && !pv_ok(mt0);
            if (__ballot(need1)) {  // rare: after st_seed / st_mt_sync / a host-written state
                // the piece first, with the counts before the spawn
                int32_t c0[7];
#pragma unroll
                for (int i = 0; i < 7; ++i) c0[i] = (int32_t)ss(ST_STAT_COUNT0 + i);
                const int pk = draw_shape<kWin, false>(need1, c0, mtst, p.mt + e0 * kMtPitch, sm.S, lane, pre, false);
                if (need1) {
                    sid = pk;
#pragma unroll
                    for (int i = 0; i < 7; ++i) cnt[i] = c0[i] + (i == pk);  // _new_piece :199
#pragma unroll
                    for (int i = 0; i < 7; ++i) csid = pk == i ? cnt[i] : csid;
                }
                dpar = draw_par(cnt);
            }
            sm.pick1[lane] = (uint32_t)sid;
            if (lane == 0) lds_flag_set(&sm.f2, (uint32_t)t + 1u);
            const uint32_t m0 = mtst;
            const int npv = draw_core<kWin>(dr_spec, dpar, mtst, p.mt + e0 * kMtPitch, sm.S, lane, pre,
                                            want_pre && pv_ok(mt0));
            mt_new = pv_pack(mtst, npv, mt_consumed(m0, mtst));
        } else {
            sm.pick1[lane] = (uint32_t)sid;
            if (lane == 0) lds_flag_set(&sm.f2, (uint32_t)t + 1u);
        }
        // this step's next-generation chunk (its operands arrived long ago);
        // its env's progress advances unless that env's own draw switched
        // generations (finishing the successor itself: same words)
        const int chunk_pg = mt_chunk_store<KSTEPS == 1 ? kST : 0>(mrs, lane, chunk);
        const bool chunk_me = lane == chunk.l;
        ST_STAMP(4);
        if constexpr (STAMP) {  // 1: a draw started a generation, 2: a draw ran past its 8 words
            const int i0 = (int)(mt_before & 0x3FFu), i1 = (int)(mt_new & 0x3FFu);
            draw_kind = (__ballot(dr_spec && i1 < i0) ? 1u : 0u) | (__ballot(dr_spec && i1 >= i0 && i1 - i0 > 8) ? 2u : 0u);
        }
        // commit: lanes whose lock consumed the preview
        bool dr = draw;
        dr = locknow;
        if (p.autoreset != ST_AUTORESET_SAME_STEP) {
            lds_flag_wait(&sm.f1, (uint32_t)t + 1u);
            const uint32_t w = lane < 32 ? sm.drawm[0] : sm.drawm[1];
            dr = (w >> (lane & 31)) & 1u;
        }
        // (a lane that locks but does not draw -- a death without auto-reset
        // -- keeps its old MT word: its speculative draw is dropped)
        uint32_t mt_out = dr ? mt_new : mt0;
        if (chunk_me && (mt_out & (1u << 20)) == (mt0 & (1u << 20))) {
            int i2, pg2, c2;
            mt_unpack(mt_out, i2, pg2, c2);
            mt_out = mt_keep(mt_out, mt_pack(i2, chunk_pg, c2));
        }
        if constexpr (STEP2) {
            // st_step: this wave's changed counter rows straight from the
            // registers, one coalesced dword per lane and row (no staging
            // through LDS at the end of the chain): the MT word, and the
            // count of the spawned shape (csid, counted above)
            const auto rs = buf_rsrc(p.stats, (uint32_t)kHotRows * (uint32_t)sd * 4u);
            const uint32_t eo = (uint32_t)e * 4u;
            // (ablation 2048: the lock-path counter stores dropped, timing only)
            const bool cst = !(kAblate & (2048u | 32768u));
            const bool mst = cst && !(kAblate & 131072u) && (dr || chunk_me);
            const bool kst = cst && !(kAblate & 65536u) && dr;
            __builtin_amdgcn_raw_buffer_store_b32(mt_out, rs, mst ? eo + (uint32_t)ST_STAT_MT_INDEX * (uint32_t)sd * 4u : kOff,
                                                  0, kST);
            __builtin_amdgcn_raw_buffer_store_b32(
                (uint32_t)csid, rs, kst ? eo + (uint32_t)(ST_STAT_COUNT0 + sid) * (uint32_t)sd * 4u : kOff, 0, kST);
            if constexpr (VEC) {  // st_step_vec's info snapshot: the shape counts after the step
                const auto ri = buf_rsrc(p.info, (uint32_t)ST_NSTAT * (uint32_t)p.n * 4u);
#pragma unroll
                for (int i = 0; i < 7; ++i)
                    __builtin_amdgcn_raw_buffer_store_b32(
                        (uint32_t)(dr ? cnt[i] : (int32_t)ss(ST_STAT_COUNT0 + i)), ri,
                        real ? ((uint32_t)(ST_STAT_COUNT0 + i) * (uint32_t)p.n + (uint32_t)e) * 4u : kOff, 0, kNT);
            }
        } else {
            // rollout: the staged rows (stored at the end of the launch)
            if (dr || chunk_me) ss(ST_STAT_MT_INDEX) = mt_out;
            if (dr) atomicAdd(&ss(ST_STAT_COUNT0 + sid), 1u);  // shape_counts[name] += 1, :199 (ds_add, no return)
            sm.mtw[t & 1][lane] = mt_out;  // the logic wave's next step reads it after B1
        }
        ST_STAMP(11);
    }

    if constexpr (DO_L) {
        // a spawn without a preview takes the draw wave's first draw (rare)
        const bool need1 = draw && !pv_ok(mt0);
        if (__ballot(need1)) {
            lds_flag_wait(&sm.f2, (uint32_t)t + 1u);
            if (need1) sid = (int)sm.pick1[lane];
        }
        ST_STAMP(4);
        uint32_t pw_out = pack_piece(id, rot, ax, ay, lock);
        if (draw) pw_out = pack_piece(sid, 0, W / 2, 0, lock);
        if (spawn) {
            odesc = tab(sid * 4);
            oax = W / 2;
            oay = 0;
        }

        // ---- counters back to the staged rows (tetris_env.py:253, :264-299) ----
        if constexpr (LCL) {
            // the late-loaded counters (issued before B1; the lock path kept
            // deltas) -- absolute values and the old ones for the dirty tests
            if (locknow) {
                o_score = (int32_t)lcv[0];
                o_lines = (int32_t)lcv[1];
                o_holes = (int32_t)lcv[2];
                o_height = (int32_t)lcv[3];
                o_deaths = (int32_t)lcv[4];
                score += o_score;
                lines += o_lines;
                deaths += o_deaths;
                if (!hset) height = o_height;
            }
        }
        [[maybe_unused]] int32_t ep_t = 0, ep_s = 0, ep_l = 0, ep_h = 0;  // VEC: info's ep_* rows
        if constexpr (VEC) {
            if (reset_now) {
                ep_t = time;
                ep_s = score;
                ep_l = lines;
                ep_h = holes;
            }
        }
        if (reset_now) {  // the finished episode's counters (ST_AUTORESET_SAME_STEP)
            int32_t *st = p.stats + e;
            st[ST_STAT_EP_TIME * sd] = time;
            st[ST_STAT_EP_SCORE * sd] = score;
            st[ST_STAT_EP_LINES * sd] = lines;
            st[ST_STAT_EP_HOLES * sd] = holes;
            time = score = lines = holes = height = 0;
        }
        // st_step stores only the counter rows that changed (per env)
        if constexpr (STEP2) {
            // st_step: straight from the registers, one coalesced dword per
            // lane and changed row (no staging through LDS at the end of the
            // chain), unconditional stores with an out-of-range offset
            // where a row did not change
            const auto rs = buf_rsrc(p.stats, (uint32_t)kHotRows * (uint32_t)sd * 4u);
            const uint32_t eo = (uint32_t)e * 4u;
            auto put = [&](int r, int32_t v, bool on) {
                __builtin_amdgcn_raw_buffer_store_b32((uint32_t)v, rs, on ? eo + (uint32_t)r * (uint32_t)sd * 4u : kOff,
                                                      0, kST);
            };
            put(ST_STAT_TIME, time, true);
            put(kPieceRow, (int32_t)pw_out, true);
            const bool cst = !(kAblate & (2048u | 16384u));  // (ablation: lock-path counter stores dropped)
            put(ST_STAT_SCORE, score, cst && locknow && score != o_score);
            put(ST_STAT_LINES, lines, cst && locknow && lines != o_lines);
            put(ST_STAT_HOLES, holes, cst && locknow && holes != o_holes);
            put(ST_STAT_PIECE_HEIGHT, height, cst && locknow && height != o_height);
            put(ST_STAT_DEATHS, deaths, cst && locknow && deaths != o_deaths);
            if constexpr (VEC) {
                // st_step_vec's info snapshot: this wave's rows for every env
                // (locking lanes from the registers, the others unchanged)
                const auto ri = buf_rsrc(p.info, (uint32_t)ST_NSTAT * (uint32_t)p.n * 4u);
                const uint32_t io = (uint32_t)e * 4u;
                auto inf = [&](int r, int32_t v) {
                    __builtin_amdgcn_raw_buffer_store_b32((uint32_t)v, ri, real ? io + (uint32_t)r * (uint32_t)p.n * 4u : kOff,
                                                          0, kNT);
                };
                inf(ST_STAT_TIME, time);
                inf(kPieceRow, (int32_t)pw_out);
                inf(ST_STAT_SCORE, locknow ? score : (int32_t)ss(ST_STAT_SCORE));
                inf(ST_STAT_LINES, locknow ? lines : (int32_t)ss(ST_STAT_LINES));
                inf(ST_STAT_HOLES, locknow ? holes : (int32_t)ss(ST_STAT_HOLES));
                inf(ST_STAT_PIECE_HEIGHT, locknow ? height : (int32_t)ss(ST_STAT_PIECE_HEIGHT));
                inf(ST_STAT_DEATHS, locknow ? deaths : (int32_t)ss(ST_STAT_DEATHS));
                inf(ST_STAT_EP_TIME, ep_t);
                inf(ST_STAT_EP_SCORE, ep_s);
                inf(ST_STAT_EP_LINES, ep_l);
                inf(ST_STAT_EP_HOLES, ep_h);
            }
        } else {
            ss(ST_STAT_TIME) = (uint32_t)time;
            ss(kPieceRow) = pw_out;
            if (locknow) {
                auto put = [&](int r, int32_t v, int32_t) { ss(r) = (uint32_t)v; };
                put(ST_STAT_SCORE, score, o_score);
                put(ST_STAT_LINES, lines, o_lines);
                put(ST_STAT_HOLES, holes, o_holes);
                put(ST_STAT_PIECE_HEIGHT, height, o_height);
                put(ST_STAT_DEATHS, deaths, o_deaths);
            }
        }

        // ---- observation (tetris_env.py:301-302): board + current piece ----
        if constexpr (KSTEPS != 1) {
            if (KSTEPS != 1 || spawn) paint<S32>(L, lane, odesc.x, odesc.y, oax, oay, hmask);
        }
        wave_sync();
        const bool wide_obs = (p.n & 3) == 0 && e0 + kWave <= p.n &&
                              (reinterpret_cast<uintptr_t>(p.obs) & 15u) == 0 &&
                              (!VEC || (reinterpret_cast<uintptr_t>(p.final_obs) & 15u) == 0);
        if (obs_t && !(kAblate & 8u)) {
            if (OVP && wide_obs) {
                // stored with the board rows
            } else if (wide_obs) {
                const uint32_t noff = (uint32_t)lrow * (uint32_t)p.n + (uint32_t)lcc;
#pragma unroll
                for (int q = 0; q < NBQ; ++q) {  // interleaved read/store (measured: reads-first
                                                 // costs the packed rollout ~7%)
                    if ((WT || 4 * q < W) && 4 * q + lrow < W) {
                        uint4 v = *reinterpret_cast<const uint4 *>(&L[(4 * q + lrow + kPad) * kWave + lcc]);
                        v.x &= hmask;
                        v.y &= hmask;
                        v.z &= hmask;
                        v.w &= hmask;
                        buf_store16<kNT>(buf_rsrc(obs_t, (uint32_t)W * (uint32_t)p.n * 4u),
                                         ((uint32_t)e0 + (uint32_t)(4 * q) * (uint32_t)p.n + noff) * 4u, v);
                    }
                }
            } else if (real) {  // ragged / unaligned: one dword per row, 32-bit offsets (SGPRs)
                const auto ro = buf_rsrc(obs_t, (uint32_t)W * (uint32_t)p.n * 4u);
                // VEC with final_obs: a reset env returns the reset obs, its
                // terminal obs goes to final_obs
                const bool fin = VEC && p.final_obs && reset_now;
                const auto rf = buf_rsrc(VEC ? p.final_obs : nullptr, (uint32_t)W * (uint32_t)p.n * 4u);
#pragma unroll 1
                for (int x = 0; x < W; ++x) {
                    const uint32_t v = (lcol(L, x, lane) | (OVP ? lcol(sm.OV, x, lane) : 0u)) & hmask;
                    const uint32_t off = ((uint32_t)x * (uint32_t)p.n + (uint32_t)e) * 4u;
                    __builtin_amdgcn_raw_buffer_store_b32(fin ? 0u : v, ro, off, 0, kNT);
                    if constexpr (VEC) __builtin_amdgcn_raw_buffer_store_b32(v, rf, fin ? off : kOff, 0, kNT);
                }
            }
        }
        if constexpr (KSTEPS == 1) {
            if (p.wire) {
                // st_step_wire (BASELINE C5's gather format, st_wire_words):
                // per env one bit stream -- column x's H obs bits at bit x*H,
                // then the reward's 32 bits (lossless: host-written counters
                // can make a penalise_*_increase reward of any int32) and done
                // -- as words [j][n], so one gather moves ceil((W*H + 33) / 32)
                // words per env (10x20: 8, 32 B) instead of obs + reward +
                // done as W + 2 words (48 B)
                const auto rw = buf_rsrc(p.wire, (uint32_t)((W * H + 33 + 31) / 32) * (uint32_t)p.n * 4u);
                uint32_t off = (uint32_t)e * 4u;
                const uint32_t rowb = (uint32_t)p.n * 4u;
                uint64_t acc = 0;
                int nb = 0;
                auto put = [&](uint32_t bits, int k) {  // k <= 32
                    acc |= (uint64_t)bits << nb;
                    nb += k;
                    if (nb >= 32) {
                        __builtin_amdgcn_raw_buffer_store_b32((uint32_t)acc, rw, real ? off : kOff, 0, kNT);
                        off += rowb;
                        acc >>= 32;
                        nb -= 32;
                    }
                };
#pragma unroll
                for (int x = 0; x < (WT ? WT : kMaxW); ++x)
                    if (WT || x < W) put((lcol(L, x, lane) | lcol(sm.OV, x, lane)) & hmask, H);
                put((uint32_t)rew, 32);
                put(died ? 1u : 0u, 1);
                if (nb > 0) __builtin_amdgcn_raw_buffer_store_b32((uint32_t)acc, rw, real ? off : kOff, 0, kNT);
            }
        }
        if (F32) {
            // float32 obs [n][W][H] of the wave's envs is one contiguous block,
            // written as lane-consecutive float4 chunks.
            const int64_t nreal64 = p.n - e0 < kWave ? p.n - e0 : kWave;
            const int nreal = (int)nreal64;
            float *out = p.obs_f32 + ((int64_t)t * p.n + e0) * (W * H);
            if constexpr (WT != 0 && HT % 4 == 0) {
                // chunk c = (env, column x, nibble q): 4 floats = bits 4q..4q+3 of
                // the column word; the float4 comes from the 16-entry table.
                constexpr int CPC = HT / 4, CPE = WT * CPC;
                uint32_t *O = sm.O;
                // (VEC with final_obs: a reset env's float32 obs is the reset obs)
                const uint32_t omask = VEC && p.final_obs && reset_now ? 0u : hmask;
#pragma unroll
                for (int x = 0; x < WT; ++x)
                    O[lane * (WT + 1) + x] = (lcol(L, x, lane) | (OVP ? lcol(sm.OV, x, lane) : 0u)) & omask;
                wave_sync();
                float4 *out4 = reinterpret_cast<float4 *>(out);
                const float4 *F4 = reinterpret_cast<const float4 *>(sm.F4);
                const int total = nreal * CPE;
                for (int c = lane; c < total; c += kWave) {
                    const int ee = c / CPE;
                    const int cr = c - ee * CPE;
                    const int x = cr / CPC;
                    const int q = cr - x * CPC;
                    const float4 f = F4[(O[ee * (WT + 1) + x] >> (4 * q)) & 15u];
                    if constexpr (KSTEPS != 1) {
                        // rollouts: non-temporal (A/B: -13% f32 rollout; the MT and
                        // state lines stay in L2 instead of the streamed obs; +7% on
                        // the single-step launch before its other stores were
                        // made nt, +-0 after, so it keeps plain stores)
                        typedef float f32x4 __attribute__((ext_vector_type(4)));
                        const f32x4 fv = {f.x, f.y, f.z, f.w};
                        __builtin_nontemporal_store(fv, reinterpret_cast<f32x4 *>(&out4[c]));
                    } else {
                        out4[c] = f;
                    }
                }
            } else {
                const int per_env = W * H;
                const int total = nreal * per_env;
                // (VEC with final_obs: KM[ee] = 0 for a reset env -- its reset obs)
                auto word = [&](int ee, int x) {
                    return (L[(x + kPad) * kWave + ee] | (OVP ? sm.OV[(x + kPad) * kWave + ee] : 0u)) &
                           (VEC && p.final_obs ? sm.KM[ee] : hmask);
                };
                for (int f = lane; f < total; f += kWave) {
                    const int ee = f / per_env;
                    const int rem = f - ee * per_env;
                    const int x = rem / H;
                    const int y = rem - x * H;
                    out[f] = (float)((word(ee, x) >> y) & 1u);
                }
            }
        }
        ST_STAMP(5);

        if constexpr (KSTEPS != 1) {
            // ---- state for the next step: board = obs minus the overlay ----
            // Erasing the overlaid piece yields the post-step board for every
            // lane: non-locking lanes and spawns (overlay cells were empty), and a
            // death without auto-reset (R8: _set_piece(False), tetris_env.py:303).
            wave_sync();
            erase<S32>(L, lane, odesc.x, odesc.y, oax, oay, hmask);
            if (reset_now)
                for (int x = 0; x < W; ++x) lcol(L, x, lane) = floorb;
        }
    }
    }  // for t
    wave_sync();
    if constexpr (ACT) {
        // st_set_action_flag's sticky word: only lanes that saw a bad action
        // store (a raw buffer store with an out-of-range offset elsewhere, no
        // branch); a null flag has an empty range, so nothing is written
        __builtin_amdgcn_raw_buffer_store_b32(1u, buf_rsrc(p.act_flag, 4u), bad_act ? 0u : kOff, 0, 0);
    }
    if constexpr (KSTEPS != 1 && DO_L) {
        // 32-bit buffer offsets: 64-bit row offsets shared with the prologue
        // would stay live (in SGPRs) across the step loop
        const auto rb = buf_rsrc(p.board, (uint32_t)((W + 3) & ~3) * (uint32_t)sd * 4u);
        const uint32_t boff = (uint32_t)e0 * 4u + loff * 4u;
#pragma unroll
        for (int q = 0; q < NBQ; ++q) {
            if (WT || 4 * q < W) {  // rows >= W: padding rows of the allocation
                uint4 v = *reinterpret_cast<const uint4 *>(&L[(4 * q + lrow + kPad) * kWave + lcc]);
                v.x &= hmask;
                v.y &= hmask;
                v.z &= hmask;
                v.w &= hmask;
                buf_store16<kST>(rb, boff + (uint32_t)(4 * q) * (uint32_t)sd * 4u, v);
            }
        }
    }
    // rollout: the staged counter rows, each wave the rows it owns (logic:
    // 0-5 and the piece row, draw: the shape counts and the MT word); st_step
    // stored its changed rows per lane above
    constexpr uint32_t kRowsD = ((1u << 7) - 1u) << ST_STAT_COUNT0 | 1u << ST_STAT_MT_INDEX;
    constexpr uint32_t kOwn = ROLE == kRoleD ? kRowsD : ((1u << kHotRows) - 1u) & ~kRowsD;
    const auto rs = buf_rsrc(p.stats, (uint32_t)kHotRows * (uint32_t)sd * 4u);
    const uint32_t soff = (uint32_t)e0 * 4u + loff * 4u;
#pragma unroll
    for (int q = 0; q < kHotQ; ++q) {
        if constexpr (STEP2) break;
        // row 15 (ep_time) is never staged: it is stored per lane on a reset
        if (((kOwn >> (4 * q)) & 0xFu) == 0u) continue;
        const bool st = (kOwn >> (4 * q + lrow)) & 1u;
        buf_store16<kST>(rs, st ? soff + (uint32_t)(4 * q) * (uint32_t)sd * 4u : kOff,
                         *reinterpret_cast<const uint4 *>(&SS[(4 * q + lrow) * kWave + lcc]));
    }
    if constexpr (STAMP && KSTEPS != 1) {
        // rollout stamp build: words [0, 16) of the workgroup's slot the
        // logic wave's per-phase cycle totals (stamp index i), [16, 32) the
        // draw wave's; word 12 / 28: s_memrealtime span, 13 / 29: steps
        ST_STAMP(6);
        uint64_t *slot = p.stamps + (int64_t)blockIdx.x * kStampWords + (ROLE == kRoleD ? 16 : 0);
        if (lane == 0) {
#pragma unroll
            for (int i = 0; i < 12; ++i) slot[i] = tacc[i];
            slot[12] = __builtin_amdgcn_s_memrealtime() - rt0;
            slot[13] = (uint64_t)K;
        }
    }
    if constexpr (STAMP && KSTEPS == 1) {
        // words [0, 16) of the workgroup's slot: the logic wave (stamps
        // 0-9, realtime start/end, HW_ID, XCC_ID, draw kind); [16, 32): the
        // draw wave (stamps 0-11, realtime start/end)
        ST_STAMP(6);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        ST_STAMP(7);
        uint64_t *slot = p.stamps + (int64_t)blockIdx.x * kStampWords + (ROLE == kRoleD ? 16 : 0);
        if (lane == 0) {
            if constexpr (ROLE == kRoleD) {
#pragma unroll
                for (int i = 0; i < 12; ++i) slot[i] = tstamp[i];
                slot[12] = rt0;
                slot[13] = __builtin_amdgcn_s_memrealtime();
                slot[14] = draw_kind;
            } else {
#pragma unroll
                for (int i = 0; i < 10; ++i) slot[i] = tstamp[i];
                slot[10] = rt0;
                slot[11] = __builtin_amdgcn_s_memrealtime();
                slot[12] = __builtin_amdgcn_s_getreg(0xF804);  // HW_ID
                slot[13] = __builtin_amdgcn_s_getreg(0xF814);  // XCC_ID
                slot[14] = tstamp[10];  // round 6: reward / done issued
                slot[15] = tstamp[11];  // round 6: the store phase's LDS reads arrived
            }
        }
    }
}

// st_step: two waves per 64 envs (kRoleL, kRoleD), see run_steps.
// What the prologue's first loads address -- the state and action
// pointers, the row stride, the env count -- comes as six leading scalar
// arguments, preloaded into SGPRs at wave launch (gfx950 kernarg preload:
// the Makefile builds with -mllvm -amdgpu-kernarg-preload-count=6; the
// code object keeps the s_load fallback for firmware without it), so those
// loads do not wait for a scalar load of the kernarg segment; the rest of
// KParams arrives by s_load meanwhile, long before it is needed.  (Round 5
// A/B, profiles/r05/ab_kernarg_preload.txt: C3 4.74 -> 4.62 us, C4 4.87 ->
// 4.75 us per graph-replayed step.)
template <int WT, int HT, bool F32, bool STAMP = false, bool SC0 = false, bool VEC = false>
__global__ __launch_bounds__(2 * kWave) void k_step(uint32_t *board, int32_t *stats, const uint8_t *actions,
                                                    uint32_t *mt, int64_t stride, int64_t n, KParams p0) {
    KParams p = p0;
    p.board = board;
    p.stats = stats;
    p.actions = actions;
    p.mt = mt;
    p.stride = stride;
    p.n = n;
    __shared__ StepLds<WT, F32, 1> sm;
    if (threadIdx.x < kWave) run_steps<WT, HT, F32, STAMP, 1, SC0, kRoleL, VEC>(p, sm);
    else run_steps<WT, HT, F32, STAMP, 1, SC0, kRoleD, VEC>(p, sm);
}

// ---------------------------------------------------------------- rollout
// st_rollout: K consecutive TetrisEngine.step calls (tetris_env.py:243-304)
// in one launch, THREE waves per 64 envs:
//   logic  (L): action + gravity + lock decision, lock path (paint, full rows,
//               compaction, holes / height, scoring, death), reward / done,
//               spawn; state in registers (piece word, clock, counters and the
//               piece's four rotation descriptors), the board in LDS;
//   draw   (D): the piece draws, TWO spawns ahead: each env's next two pieces
//               (q0 = the preview of the state word, q1 = the one after it)
//               sit in a per-lane LDS ring; a round s refills the pieces the
//               logic wave's step s consumed.  The piece sequence does not
//               depend on the actions (clear() keeps the shape counts,
//               tetris_env.py:306-315; counts change only at spawns, :199),
//               so q1 is drawn with the counts after q0's spawn, exactly the
//               ones the reference's _choose_shape will see.  MT words come
//               from a 16-word register window per lane (draw_win), reloaded
//               after each draw and merged one round later, so no draw waits
//               for memory; shape counts and MT positions in registers; the
//               next-generation chunk;
//   output (O): the observation of every step -- the board plane OR'ed with
//               an overlay plane OV the logic wave writes (the current piece's
//               cells, or for an env reset in this step its whole terminal
//               board) -- packed and float32 stores, then OV cleared.
// No barrier inside the step loop: the three waves run their own chains and
// meet only through progress counters in LDS (each written by one wave, each
// wait one-way): fl = t + 1 once the logic wave's consumption mask of step t
// is in cm[t & 1]; fd = s + 2 once draw round s wrote its pieces (1 after the
// two initial draws); fo = t + 1 once step t's planes are final; fq = t + 1
// once the output wave has read them.  The logic wave's step t needs round
// t - 2 (fd >= t: a piece consumed at step t was drawn when the piece two
// before it was consumed, at step <= t - 2) and the output of step t - 1
// (fq >= t, before it changes a plane); the draw wave's round s needs fl >=
// s + 1.  So the draw chain runs up to ~2 steps behind the logic chain and a
// step takes the longer of the two, not their sum: round 3's B1 per step made
// the logic wave wait ~1,400 of ~4,450 cycles for the draw wave's previous
// step (tools/ro_stamps.py, profiles/r03/ro_stamps_3wave_fine.txt).
// At the end, the committed state is q0's (the state word's preview and the
// MT position after its draw); q1's draw is dropped, and st_mt_sync's rewind
// rule is unchanged.  The next-generation chunk is built only for envs whose
// reference state (before q0's draw) is in the generation q1 ended in, so it
// never overwrites words a committed preview may give back.
constexpr int kRoleO = 3;
// issue priority of the rollout's logic wave (its chain sets the step: 3
// against 0, -6% per step; logic 0-3 x draw 0-2 measured in round 3,
// profiles/r03/ro_ab_priorities.txt); the draw wave runs at kDrawPrio after
// its first round, the output wave at 0
constexpr int kRoLogicPrio = 3;
template <int WT, bool F32>
struct RoLds {
    static constexpr int kCols = (WT ? WT : kMaxW) + 2 * kPad;
    uint32_t L[kCols * kWave] __attribute__((aligned(16)));   // board columns, walls at both ends
    uint32_t OV[kCols * kWave] __attribute__((aligned(16)));  // obs overlay plane (walls never set)
    uint32_t SS[kHotQ * 4 * kWave] __attribute__((aligned(16)));  // staged counter rows (prologue / epilogue)
    uint32_t T2[2 * 28] __attribute__((aligned(8)));              // piece table {m, g}
    uint32_t S[kMtN];                                             // mt_finish scratch
    uint32_t O[F32 ? kWave * (kMaxW + 1) : 1];                    // float32 writer staging
    float F4[F32 ? 64 : 4] __attribute__((aligned(16)));
    uint32_t qring[kWave];  // per lane: the env's i-th queued piece in bits 4 (i & 3) .. (draw -> logic)
    uint32_t cm[2][2];      // step t's consumption mask (a spawn or a same-step reset) in cm[t & 1]
    uint32_t act[4][kWave];  // step t's actions in act[t & 3] (draw -> logic, four steps ahead)
    uint32_t rw[2][kWave], dn[2][kWave];  // step t's reward / done in [t & 1] (logic -> output)
    uint32_t ep[2][4][kWave];             // a same-step reset's episode time / score / lines / holes
    // packed obs (the output wave builds the next-generation chunks):
    uint32_t cw[kWave];   // per lane: chunk candidate << 31 | cur << 10 | pg (draw -> output)
    uint32_t cpg[kWave];  // per lane: valid << 31 | cur << 10 | pg after a chunk (output -> draw)
    uint32_t fl, fd, fo, fq;  // progress counters (see above)
};
// d[r] by selects on values (a select between two array elements would be
// a pointer select, which puts the array in scratch memory)
__device__ __forceinline__ uint2 sel4(const uint2 (&d)[4], int r) {
    const bool b0 = r & 1, b1 = r & 2;
    const uint32_t ax = b0 ? d[1].x : d[0].x, ay = b0 ? d[1].y : d[0].y;
    const uint32_t bx = b0 ? d[3].x : d[2].x, by = b0 ? d[3].y : d[2].y;
    return make_uint2(b1 ? bx : ax, b1 ? by : ay);
}

template <int WT, int HT, bool F32, bool SC0, bool STAMP, int ROLE>
__device__ __forceinline__ void rollout_wave(const KParams &p, RoLds<WT, F32> &sm) {
    constexpr bool S32 = HT != 0 && HT <= 25;  // see pc_bits
    // the next-generation chunks: built by the output wave with packed obs
    // (it idles most of a step), by the draw wave with float32 obs (the
    // output wave's stores set that step)
    constexpr bool CHO = !F32;
    const uint32_t kFlags = SC0 ? (p.flags & (ST_REWARD_STEP | ST_STEP_RESET)) : p.flags;
#if defined(ST_ABLATION) && ST_ABLATION
    const uint32_t kAblate = p.ablate;
#else
    constexpr uint32_t kAblate = 0u;
#endif
    // diagnostic build: per-phase cycle totals over the launch (stamp index i
    // = the phase that ends there), words [16 * role, 16 * role + 12) of the
    // workgroup's slot, + s_memrealtime span and the step count
    [[maybe_unused]] uint32_t tacc[12] = {};
    [[maybe_unused]] uint64_t tlast = 0, rt0 = 0;
    auto stamp = [&](int i) {
        if constexpr (STAMP) {
            __builtin_amdgcn_sched_barrier(0);
            const uint64_t now = __builtin_amdgcn_s_memtime();
            tacc[i] += (uint32_t)(now - tlast);
            tlast = now;
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    if constexpr (STAMP) {
        rt0 = __builtin_amdgcn_s_memrealtime();
        tlast = __builtin_amdgcn_s_memtime();
    }
    uint32_t *const L = sm.L;
    uint32_t *const OV = sm.OV;
    uint32_t *const SS = sm.SS;
    const int W = WT ? WT : p.W;
    const int H = HT ? HT : p.H;
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t e0 = (int64_t)blockIdx.x * kWave;
    const int64_t e = e0 + lane;
    const int64_t sd = p.stride;
    const bool real = e < p.n;
    const uint32_t hmask = (1u << H) - 1u;
    const uint32_t floorb = ~hmask;
    const int K = p.k;
    const int lrow = lane >> 4, lcc = 4 * (lane & 15);  // transposed 16-B slot: row-in-group, env
    constexpr int NBQ = ((WT ? WT : kMaxW) + 3) / 4;
    const uint32_t loff = (uint32_t)lrow * (uint32_t)sd + 4u * (uint32_t)(lane & 15);
    auto clamp_off = [&](int q, int nrows) -> uint32_t {
        const int r = 4 * q + lrow < nrows ? lrow : nrows - 1 - 4 * q;
        return (uint32_t)r * (uint32_t)sd + 4u * (uint32_t)(lane & 15);
    };
    auto ss = [&](int r) -> uint32_t & { return SS[r * kWave + lane]; };
    auto tab = [&](int i) -> uint2 { return *reinterpret_cast<const uint2 *>(&sm.T2[2 * i]); };
    auto col = [&](uint32_t *P, int x) -> uint32_t & { return P[(x + kPad) * kWave + lane]; };

    // ---- prologue: state into LDS (16 B per lane, transposed), B0 ----
    // logic: board + counter groups 0-1 (time .. count1); draw: counter
    // groups 2-3 (count2 .. MT word, piece), the walls, the piece table;
    // output: the zeroed overlay plane
    const uint32_t *bsrc = p.board + e0;
    const uint32_t *ssrc = reinterpret_cast<const uint32_t *>(p.stats) + e0;
    if constexpr (ROLE == kRoleL) {
        uint4 bv[NBQ], sv[2];
#pragma unroll
        for (int q = 0; q < NBQ; ++q)
            if (WT || 4 * q < W)
                bv[q] = *reinterpret_cast<const uint4 *>(bsrc + (size_t)(4 * q) * sd +
                                                         (4 * q + 4 <= W ? loff : clamp_off(q, W)));
#pragma unroll
        for (int q = 0; q < 2; ++q) sv[q] = *reinterpret_cast<const uint4 *>(ssrc + (size_t)(4 * q) * sd + loff);
#pragma unroll
        for (int q = 0; q < NBQ; ++q) {
            if (WT || 4 * q < W) {
                uint4 v = bv[q];
                v.x |= floorb;
                v.y |= floorb;
                v.z |= floorb;
                v.w |= floorb;
                // rows >= W (allocation padding) are not staged (the draw
                // wave writes the wall columns in the same prologue)
                if (4 * q + lrow < W) *reinterpret_cast<uint4 *>(&L[(4 * q + lrow + kPad) * kWave + lcc]) = v;
            }
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) *reinterpret_cast<uint4 *>(&SS[(4 * q + lrow) * kWave + lcc]) = sv[q];
        if (lane == 0) sm.fo = 0u;
    } else if constexpr (ROLE == kRoleD) {
        uint4 sv[2];
#pragma unroll
        for (int q = 2; q < kHotQ; ++q)
            sv[q - 2] = *reinterpret_cast<const uint4 *>(ssrc + (size_t)(4 * q) * sd +
                                                         (4 * q + 4 <= kHotRows ? loff : clamp_off(q, kHotRows)));
        uint32_t tab_m = 0, tab_g = 0;
#pragma unroll
        for (int i = 0; i < 28; ++i) {
            asm("v_writelane_b32 %0, %1, %2" : "+v"(tab_m) : "s"(kBox.m[i]), "i"(i));
            asm("v_writelane_b32 %0, %1, %2" : "+v"(tab_g) : "s"(kBox.g[i]), "i"(i));
        }
#pragma unroll
        for (int x = 0; x < kPad; ++x) {
            L[x * kWave + lane] = ~0u;
            L[(W + kPad + x) * kWave + lane] = ~0u;
        }
        if (lane < 28) {
            sm.T2[2 * lane] = tab_m;
            sm.T2[2 * lane + 1] = tab_g;
        }
        if constexpr (F32) {
            if (lane < 16) {
                sm.F4[4 * lane] = (float)(lane & 1);
                sm.F4[4 * lane + 1] = (float)((lane >> 1) & 1);
                sm.F4[4 * lane + 2] = (float)((lane >> 2) & 1);
                sm.F4[4 * lane + 3] = (float)((lane >> 3) & 1);
            }
        }
#pragma unroll
        for (int q = 2; q < kHotQ; ++q) *reinterpret_cast<uint4 *>(&SS[(4 * q + lrow) * kWave + lcc]) = sv[q - 2];
        if (lane == 0) {
            sm.fl = 0u;
            sm.fd = 0u;
            sm.fq = 0u;
        }
        sm.cw[lane] = 0u;
    } else {
        for (int i = lane; i < RoLds<WT, F32>::kCols * kWave; i += kWave) OV[i] = 0u;
        sm.cpg[lane] = 0u;
    }
    wg_barrier();  // B0
    stamp(0);
    if constexpr (ROLE == kRoleL) __builtin_amdgcn_s_setprio(kRoLogicPrio);

    if constexpr (ROLE == kRoleL) {
        // ================================================================ logic
        uint32_t pw = ss(kPieceRow);
        int32_t time = (int32_t)ss(ST_STAT_TIME);
        int32_t score = (int32_t)ss(ST_STAT_SCORE), lines = (int32_t)ss(ST_STAT_LINES);
        int32_t holes = (int32_t)ss(ST_STAT_HOLES), height = (int32_t)ss(ST_STAT_PIECE_HEIGHT);
        int32_t deaths = (int32_t)ss(ST_STAT_DEATHS);
        uint2 d4[4];  // the current piece's four rotations
#pragma unroll
        for (int r = 0; r < 4; ++r) d4[r] = tab((int)(pw & 7u) * 4 + r);
        bool bad_act = false;
        // LAZYH (fixed width): holes is counted when read -- a death, a holes
        // reward, the epilogue -- not at every lock (the board changes only
        // at locks, clears and resets, so the epilogue's count of the final
        // board equals the count at the last lock); hstale: a lock since
        constexpr bool LAZYH = WT != 0;
        bool hstale = false;
        uint32_t nq = 0;  // pieces this env consumed so far (its next spawn: ring slot nq & 3)
        // The actions come from the ring the draw wave fills four steps ahead
        // (at the end of round t - 4, or its initial loads for t < 4, published
        // by round t - 3's fd): LDS reads, no memory wait on this chain (CDNA
        // counts loads and stores in one in-order vmcnt: a load here waited
        // for the previous step's stores as well).  Step t + 1's is read in
        // step t right after the queue wait (fd >= t covers it), so a step
        // starts with its action in a register: no poll, no LDS round trip.
        lds_flag_wait_ge(&sm.fd, 1u);
        uint32_t act_n = sm.act[0][lane];
        // the piece word's fields live in registers across steps (packed only
        // where it is published and stored)
        int pid = (int)(pw & 7u), prot = (int)((pw >> 3) & 3u), pax = (int)((pw >> 5) & 63u),
            pay = (int)((pw >> 11) & 63u), plock = (int)(pw >> 17);
        // the current rotation's descriptor, carried across
        // steps (set where the rotation or the piece changes)
        uint2 pdesc = sel4(d4, prot);
        for (int t = 0; t < K; ++t) {
            const uint32_t act = real ? act_n : 6u;
            bad_act |= act > 6u;
            int rot = prot;
            int ax = pax;
            int ay = pay;
            int lock = plock;
            stamp(1);
            // ---- action (tetris_env.py:245; value_action_map :152-160) + drop ----
            // both descriptors from registers: the columns are one LDS round trip
            const bool tries = act == 0u || act == 1u || act == 4u || act == 5u;
            const int cx = ax + (act == 0u ? -1 : (act == 1u ? 1 : 0));
            const int cr = (rot + (act == 4u ? 1 : 0) + (act == 5u ? 3 : 0)) & 3;  // (selects: the ternary chain became an exec-mask branch)
            uint2 desc = pdesc;
            const uint2 cdesc = sel4(d4, cr);
            uint32_t cur[4], cand[4];
            read_box(L, lane, desc.y, ax, cur);
            read_box(L, lane, cdesc.y, cx, cand);
            // the queue / planes hand-off, read optimistically in the same
            // LDS round trip as the columns: both counters, step t + 1's
            // action and the queue word; taken after the action phase if
            // the counters allow it, else polled there (round 4: one LDS
            // round trip less per step when the other waves are ahead;
            // 65,536 envs 1.389 -> 1.382 us/step over 3 alternating rounds,
            // profiles/r04/ab_colbatch_earlyq.txt)
            const uint32_t fdv0 = lds_flag_get(&sm.fd), fqv0 = lds_flag_get(&sm.fq);
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
            const uint32_t act_n0 = lds_ld(&sm.act[(t + 1) & 3][lane]);
            const uint32_t qwd0 = lds_ld(&sm.qring[lane]);
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
            const bool ok = tries && !collides_v<S32>(cdesc.x, ay, cand);
            ax = ok ? cx : ax;
            rot = ok ? cr : rot;
            desc.x = ok ? cdesc.x : desc.x;
            desc.y = ok ? cdesc.y : desc.y;
#pragma unroll
            for (int j = 0; j < 4; ++j) cur[j] = ok ? cand[j] : cur[j];
            int d = drop_box(desc.y, ay, cur);
            if (act == 2u) {                  // hard_drop :54-59
                ay += d;
                d = 0;
            } else if (act == 3u && d > 0) {  // soft_drop :49-51
                ay += 1;
                d -= 1;
            }
            // ---- gravity + lock delay (tetris_env.py:247-262) ----
            if (d > 0) {
                ay += 1;
                d -= 1;
                if (kFlags & ST_STEP_RESET) lock = 0;
            }
            time += 1;
            int32_t rew = (kFlags & ST_REWARD_STEP) ? 1 : 0;
            bool locknow = false;
            if (d == 0) {
                const int l1 = lock + 1;
                lock = lock_next(l1, p.lock_mod);
                locknow = lock == 0 && !(kAblate & 1u);
            }
            stamp(2);
            // the next spawn's piece (drawn by round t - 2 at the latest; the
            // two initial draws count as one round) and its descriptors, for a
            // spawn below (read under the lock path); then the output wave's
            // reads of step t - 1's planes, before this step changes them
            // both counters and the ring words they guard in one LDS round
            // trip (the writers store the data before the counters; see the
            // draw wave's mask wait): step t + 1's action (a stale row past
            // the last step: unused) and the queue word
            uint32_t qwd;
            const uint32_t need_d = t > 1 ? (uint32_t)t : 1u;
            if (((kAblate & 160u) || (int32_t)(fdv0 - need_d) >= 0) &&
                ((kAblate & 288u) || (int32_t)(fqv0 - (uint32_t)t) >= 0)) {
                act_n = act_n0;
                qwd = qwd0;
            } else {
                for (;;) {
                    const uint32_t fdv = lds_flag_get(&sm.fd), fqv = lds_flag_get(&sm.fq);
                    __atomic_signal_fence(__ATOMIC_SEQ_CST);
                    act_n = lds_ld(&sm.act[(t + 1) & 3][lane]);
                    qwd = lds_ld(&sm.qring[lane]);
                    __atomic_signal_fence(__ATOMIC_SEQ_CST);
                    const bool ok_d = (kAblate & 160u) || (int32_t)(fdv - need_d) >= 0;
                    const bool ok_q = (kAblate & 288u) || (int32_t)(fqv - (uint32_t)t) >= 0;
                    if (ok_d && ok_q) break;
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            const int sid = (int)((qwd >> (4u * (nq & 3u))) & 7u);
            uint2 s4[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) s4[r] = tab(sid * 4 + r);
            stamp(3);

            // ---- lock path (tetris_env.py:263-299) ----
            bool died = false, spawn = false;
            [[maybe_unused]] uint32_t tb[WT ? WT : 1];  // the board after the lock (a reset copies it to OV)
            if (locknow) {
                paint_box<S32>(L, lane, desc.x, desc.y, ax, ay, hmask);
                uint32_t andv = ~0u, orv = 0, sctz = 0, spop = 0;
                if constexpr (WT != 0) {
                    // all column reads before any use: one LDS round trip (see
                    // run_steps' lock path)
#pragma unroll
                    for (int x = 0; x < WT; ++x) tb[x] = col(L, x);
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int x = 0; x < WT; ++x) {
                        const uint32_t v = tb[x];
                        andv &= v;
                        orv |= v;
                        if constexpr (!LAZYH) {
                            sctz += __builtin_ctz(v);
                            spop += __builtin_popcount(v);
                        }
                    }
                } else {
#pragma unroll 8
                    for (int x = 0; x < W; ++x) {
                        const uint32_t v = col(L, x);
                        andv &= v;
                        orv |= v;
                        sctz += __builtin_ctz(v);
                        spop += __builtin_popcount(v);
                    }
                }
                andv &= hmask;
                int32_t ncl = 0;
                if (andv) {  // full rows: compact, recount (_clear_lines :205-216)
                    ncl = __builtin_popcount(andv);
                    orv = 0;
                    sctz = spop = 0;
                    if constexpr (WT != 0) {
                        uint32_t c[WT];
#pragma unroll
                        for (int x = 0; x < WT; ++x) c[x] = tb[x] & hmask;
                        uint32_t full = andv;
                        while (full) {
                            const int r = __builtin_ctz(full);
                            full &= full - 1u;
                            const uint32_t above = (1u << r) - 1u;
                            const uint32_t keep = ~(above | (1u << r));
#pragma unroll
                            for (int x = 0; x < WT; ++x) c[x] = (c[x] & keep) | ((c[x] & above) << 1);
                        }
#pragma unroll
                        for (int x = 0; x < WT; ++x) {
                            const uint32_t v = c[x] | floorb;
                            tb[x] = v;
                            col(L, x) = v;
                            orv |= v;
                            if constexpr (!LAZYH) {
                                sctz += __builtin_ctz(v);
                                spop += __builtin_popcount(v);
                            }
                        }
                    } else {
#pragma unroll 8
                        for (int x = 0; x < W; ++x) {
                            const uint32_t v = compact(col(L, x) & hmask, andv) | floorb;
                            col(L, x) = v;
                            orv |= v;
                            sctz += __builtin_ctz(v);
                            spop += __builtin_popcount(v);
                        }
                    }
                    lines += ncl;
                }
                orv &= hmask;
                // _count_holes :218-220 (LAZYH: from tb where it is needed)
                const auto count_holes = [&]() -> int32_t {
                    if constexpr (LAZYH) {
                        uint32_t hc = 0, hp = 0;
#pragma unroll
                        for (int x = 0; x < (WT ? WT : 1); ++x) {
                            hc += __builtin_ctz(tb[x]);
                            hp += __builtin_popcount(tb[x]);
                        }
                        sctz = hc;
                        spop = hp;
                    }
                    return W * H - (int32_t)sctz - ((int32_t)spop - W * (32 - H));
                };
                if (kFlags & ST_ADVANCED_CLEARS) {  // :266-269
                    constexpr uint64_t kClr = (40ull << 12) | (100ull << 24) | (300ull << 36) | (1200ull << 48);
                    const int32_t sc = ncl <= 4 ? (int32_t)((kClr >> (12 * ncl)) & 0xFFFu) : 0;
                    rew += (sc * 5) / 2;
                    score += sc;
                } else if (kFlags & ST_HIGH_SCORING) {  // :270-272
                    rew += 1000 * ncl;
                    score += ncl;
                } else {  // :273-275
                    rew += 100 * ncl;
                    score += ncl;
                }
                if (orv & 1u) {  // death :277-281
                    holes = count_holes();
                    hstale = false;
                    deaths += 1;
                    died = true;
                    rew = -100;
                } else {  // :283-299
                    const int32_t old_holes = holes;
                    // holes feeds the reward only under the two holes flags;
                    // otherwise it is recounted from the board where it is
                    // read next (a death, the epilogue)
                    if (!LAZYH || (kFlags & (ST_PENALISE_HOLES | ST_PENALISE_HOLES_INCREASE))) holes = count_holes();
                    else hstale = true;
                    const int32_t hgt = __builtin_popcount(orv);
                    if (kFlags & ST_PENALISE_HEIGHT) {
                        rew -= hgt;
                    } else if (kFlags & ST_PENALISE_HEIGHT_INCREASE) {
                        if (hgt > height) rew -= 10 * (hgt - height);
                        height = hgt;
                    }
                    if (kFlags & ST_PENALISE_HOLES) rew -= 5 * holes;
                    else if (kFlags & ST_PENALISE_HOLES_INCREASE) rew -= 5 * (holes - old_holes);
                    spawn = true;
                }
            }
            stamp(4);
            const bool reset_now = died && p.autoreset == ST_AUTORESET_SAME_STEP;
            // the lock consumed the queue's head (a death without auto-reset
            // keeps it for the next st_reset)
            const bool draw = spawn || reset_now;
            {
                const uint64_t m = __ballot(draw);
                if (lane == 0) {
                    lds_st(&sm.cm[t & 1][0], (uint32_t)m);
                    lds_st(&sm.cm[t & 1][1], (uint32_t)(m >> 32));
                    lds_flag_set(&sm.fl, (uint32_t)t + 1u);
                }
            }
            nq += draw ? 1u : 0u;
            // reward / done (and below a reset's episode counters) go to the
            // output wave through LDS (step parity t & 1; it stores them with
            // the obs): memory stores cost this chain ~2.5%, LDS writes less
            sm.rw[t & 1][lane] = (uint32_t)rew;
            sm.dn[t & 1][lane] = died ? 1u : 0u;
            stamp(5);
            // ---- this step's obs (tetris_env.py:301-302) for the output wave ----
            // a death without auto-reset: the board loses the piece (R8,
            // _set_piece(False), :303), the obs keeps it (overlay); a death
            // with auto-reset: the obs is the whole terminal board (overlay
            // plane), the board becomes empty (clear(), :306-315)
            if (died && !reset_now) erase_box<S32>(L, lane, desc.x, desc.y, ax, ay, hmask);
            const uint2 od = make_uint2(spawn ? s4[0].x : desc.x, spawn ? s4[0].y : desc.y);
            const int oax = spawn ? W / 2 : ax, oay = spawn ? 0 : ay;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int ox = box_x0(od.y, oax) + j;
                OV[(ox + kPad) * kWave + lane] = pc_bits<S32>(od.x, j, oay) & hmask;
            }
            if (reset_now) {
                if constexpr (WT != 0) {
#pragma unroll
                    for (int x = 0; x < WT; ++x) {
                        col(OV, x) = tb[x] & hmask;
                        col(L, x) = floorb;
                    }
                } else {
                    for (int x = 0; x < W; ++x) {
                        col(OV, x) = col(L, x) & hmask;
                        col(L, x) = floorb;
                    }
                }
            }
            if (reset_now) {
                // the finished episode's counters (ST_AUTORESET_SAME_STEP),
                // stored by the output wave where done is set
                sm.ep[t & 1][0][lane] = (uint32_t)time;
                sm.ep[t & 1][1][lane] = (uint32_t)score;
                sm.ep[t & 1][2][lane] = (uint32_t)lines;
                sm.ep[t & 1][3][lane] = (uint32_t)holes;
                time = score = lines = holes = height = 0;
                hstale = false;
            }
            // ---- state for the next step ----
            pid = draw ? sid : pid;
            prot = draw ? 0 : rot;
            pax = draw ? W / 2 : ax;
            pay = draw ? 0 : ay;
            plock = lock;
            pdesc.x = draw ? s4[0].x : desc.x;
            pdesc.y = draw ? s4[0].y : desc.y;
            if (lane == 0) lds_flag_set(&sm.fo, (uint32_t)t + 1u);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                d4[r].x = draw ? s4[r].x : d4[r].x;
                d4[r].y = draw ? s4[r].y : d4[r].y;
            }
            stamp(6);
        }
        wg_barrier();  // the output wave has read the last step's planes
        // ---- epilogue: board and the rows this wave owns ----
        __builtin_amdgcn_raw_buffer_store_b32(1u, buf_rsrc(p.act_flag, 4u), bad_act ? 0u : kOff, 0, 0);
        ss(ST_STAT_TIME) = (uint32_t)time;
        ss(ST_STAT_SCORE) = (uint32_t)score;
        ss(ST_STAT_LINES) = (uint32_t)lines;
        if constexpr (LAZYH) {
            if (hstale) {
                uint32_t hc = 0, hp = 0;
#pragma unroll
                for (int x = 0; x < (WT ? WT : 1); ++x) {
                    const uint32_t v = col(L, x);
                    hc += __builtin_ctz(v);
                    hp += __builtin_popcount(v);
                }
                holes = W * H - (int32_t)hc - ((int32_t)hp - W * (32 - H));
            }
        }
        ss(ST_STAT_HOLES) = (uint32_t)holes;
        ss(ST_STAT_PIECE_HEIGHT) = (uint32_t)height;
        ss(ST_STAT_DEATHS) = (uint32_t)deaths;
        ss(kPieceRow) = pack_piece(pid, prot, pax, pay, plock);
        wave_sync();
        const auto rb = buf_rsrc(p.board, (uint32_t)((W + 3) & ~3) * (uint32_t)sd * 4u);
        const uint32_t boff = (uint32_t)e0 * 4u + loff * 4u;
#pragma unroll
        for (int q = 0; q < NBQ; ++q) {
            if ((WT || 4 * q < W) && 4 * q + lrow < W) {
                uint4 v = *reinterpret_cast<const uint4 *>(&L[(4 * q + lrow + kPad) * kWave + lcc]);
                v.x &= hmask;
                v.y &= hmask;
                v.z &= hmask;
                v.w &= hmask;
                buf_store16<kST>(rb, boff + (uint32_t)(4 * q) * (uint32_t)sd * 4u, v);
            }
        }
    } else if constexpr (ROLE == kRoleD) {
        // ================================================================ draw
        uint32_t *const mtg = p.mt + e0 * kMtPitch;
        const MtRes mrs = mt_res(mtg, lane);
        const uint32_t w0 = ss(ST_STAT_MT_INDEX);
        int32_t cnt_r[7];  // shape_counts (the spawned pieces only)
#pragma unroll
        for (int i = 0; i < 7; ++i) cnt_r[i] = (int32_t)ss(ST_STAT_COUNT0 + i);
        // mtc: the committed state word (the queue head q0 as its preview, the
        // MT position after q0's draw); mta: the MT position after the last
        // queued draw (q1's), c1 the words that draw consumed
        uint32_t mtc = w0, mta = w0 & kMtLow, c1 = 0;
        // the register window: words from where it was loaded, o consumed,
        // wlim valid; wn: the next window, loaded after a lane's draw and
        // merged at the end of the following round (o_rl: o at its load)
        // the logic wave's actions, four steps ahead: loaded at the start of
        // round s, written at its end (after the window merge, which waits
        // for the loads issued before them anyway), published by round s +
        // 1's fd (no branch around a load: steps >= K read nothing)
        auto act_at = [&](int t) -> uint32_t {
            const bool in = t < K;  // wave-uniform (a per-lane resource base makes a waterfall loop)
            return __builtin_amdgcn_raw_buffer_load_b8(buf_rsrc(p.actions + (int64_t)(in ? t : 0) * p.n, (uint32_t)p.n),
                                                       in && real ? (uint32_t)e : kOff, 0, 0);
        };
        const uint32_t a0 = act_at(0), a1 = act_at(1), a2 = act_at(2), a3 = act_at(3);
        MtPre win, wn = {};
        int o = 0, wlim = win_lim(mta), o_rl = 0, wlim_n = 0;
        mt_pre_load<kMtWin>(mrs, mta, real, win);
        mt_win_consume<kMtWin>(win);
        int q0 = pv_id(w0), q1;
        {
            // the queue's two pieces: q0 where the state has no preview
            // (st_seed / st_mt_sync / a host-written state), then q1 with the
            // counts after q0's spawn
            const bool need1 = real && !pv_ok(w0);
            if (__ballot(need1)) {
                const int pk = draw_win<CHO>(need1, cnt_r, mta, win, o, wlim, mtg, sm.S, lane);
                if (need1) q0 = pk;
            }
            int32_t cq[7];
#pragma unroll
            for (int i = 0; i < 7; ++i) cq[i] = cnt_r[i] + (i == q0);
            const uint32_t m0 = mta;
            q1 = draw_win<CHO>(real, cq, mta, win, o, wlim, mtg, sm.S, lane);
            c1 = mt_consumed(m0, mta);
        }
        int32_t cq[7];  // shape counts once the queue's head has spawned
#pragma unroll
        for (int i = 0; i < 7; ++i) cq[i] = cnt_r[i] + (i == q0);
        uint32_t qw = (uint32_t)q0 | ((uint32_t)q1 << 4), nd = 2;  // the ring word, pieces drawn
        sm.qring[lane] = qw;
        sm.act[0][lane] = a0;
        sm.act[1][lane] = a1;
        sm.act[2][lane] = a2;
        sm.act[3][lane] = a3;
        if (lane == 0) lds_flag_set(&sm.fd, 1u);
        __builtin_amdgcn_s_setprio(kDrawPrio);
        bool rl = false;  // wn holds a reload to merge
        for (int s = 0; s < K; ++s) {
            stamp(1);
            // this round's next-generation chunk, for an env whose reference
            // state (before q0's draw; q0's draw straddled index 624 when idx
            // <= c) lies in the generation mta is in: operands issued first
            const uint32_t an = act_at(s + 4);
            // the env's reference generation (the state before q0's draw;
            // q0's draw straddled index 624 when idx <= c)
            auto ref_cur = [&]() {
                int ic, pgc, cc;
                mt_unpack(mtc, ic, pgc, cc);
                return cc ^ (pv_ok(mtc) && ic <= (int)((mtc >> 25) & kPvCMax) ? 1 : 0);
            };
            [[maybe_unused]] MtChunk chunk;
            // the output wave's finished chunks, read now and applied after
            // the draw (the read's latency off this chain; a progress one
            // round staler only means a rarer, same-valued mt_finish)
            [[maybe_unused]] uint32_t cpgv = 0;
            // the chunk bookkeeping (progress merge, candidacy) every other
            // round: the output wave builds a chunk every other step (round
            // 5: -1%, profiles/r05/ab_rollout_bookkeeping_every_other_round.txt)
            [[maybe_unused]] const bool cwr = !(s & 1);
            if constexpr (CHO) {
                if (cwr) cpgv = sm.cpg[lane];
            } else {
                mt_chunk_issue(mrs, mta, real && ref_cur() == (int)((mta >> 20) & 1u) && !(kAblate & 16u), lane,
                               chunk);
            }
            // the counter and the mask it guards in one LDS round trip: a
            // wave's LDS accesses execute in order and the logic wave writes
            // the mask before the counter, so a mask read issued right after
            // a counter read that passes is current (only the compiler must
            // not reorder them: a signal fence, no wait)
            uint32_t w;
            for (;;) {
                const uint32_t f = lds_flag_get(&sm.fl);
                __atomic_signal_fence(__ATOMIC_SEQ_CST);
                w = lds_ld(&sm.cm[s & 1][lane < 32 ? 0 : 1]);
                __atomic_signal_fence(__ATOMIC_SEQ_CST);
                if ((int32_t)(f - ((uint32_t)s + 1u)) >= 0) break;
                __builtin_amdgcn_s_sleep(1);
            }
            stamp(2);
            const bool cons = real && ((w >> (lane & 31)) & 1u) && !(kAblate & 2u);
            // step s consumed q0: count it (_new_piece :199), commit q1 as the
            // preview, draw the piece after it
            // (cq = the spawned pieces' counts + the head's, kept across
            // rounds: a spawn adds the new head q1's; the spawned counts
            // alone are derived once, at the end)
            if (cons) {
                mtc = pv_pack(mta, q1, c1);
                q0 = q1;
            }
            {
                const uint32_t oh = cons ? 1u << q0 : 0u;  // one bfe + add per shape
#pragma unroll
                for (int i = 0; i < 7; ++i) cq[i] += (int32_t)((oh >> i) & 1u);
            }
            const uint32_t m0 = mta;
            const int pk = draw_win<CHO>(cons, cq, mta, win, o, wlim, mtg, sm.S, lane);
            stamp(5);
            if (cons) {
                q1 = pk;
                c1 = mt_consumed(m0, mta);
                const uint32_t sh = 4u * (nd & 3u);
                qw = (qw & ~(0xFu << sh)) | ((uint32_t)pk << sh);
                nd += 1u;
            }
            lds_st(&sm.qring[lane], qw);
            if (lane == 0) lds_flag_set_inorder(&sm.fd, (uint32_t)s + 2u);
            stamp(3);
            [[maybe_unused]] int chunk_pg = 0;
            if constexpr (CHO) {
              if (cwr) {
                // the progress, where the generation is still the one the
                // chunk was built for
                int ia, pga, ca;
                mt_unpack(mta, ia, pga, ca);
                if ((cpgv >> 31) && (int)((cpgv >> 10) & 1u) == ca && (int)(cpgv & 0x3FFu) > pga) {
                    pga = (int)(cpgv & 0x3FFu);
                    mta = mt_pack(ia, pga, ca);
                }
                // this env's chunk candidacy for the output wave: the
                // reference state in the generation mta is in, successor
                // incomplete
                const bool cand = real && ref_cur() == ca && pga < kMtN && !(kAblate & 16u);
                sm.cw[lane] = (cand ? 0x80000000u : 0u) | ((uint32_t)ca << 10) | (uint32_t)pga;
              }
            } else {
                chunk_pg = mt_chunk_store<0>(mrs, lane, chunk);
            }
            // windows: merge the reload of the previous round, reload where
            // this round drew (valid words by the progress before this
            // round's chunk: conservative)
            stamp(6);
            mt_win_consume<kMtWin>(wn);
            stamp(7);
            if (rl) {
#pragma unroll
                for (int j = 0; j < kMtWin; ++j) win.w[j] = wn.w[j];
                o -= o_rl;
                wlim = wlim_n;
            }
            rl = cons;
            lds_st(&sm.act[s & 3][lane], an);  // step s + 4's (the logic wave has read step s's)
            mt_pre_load<kMtWin>(mrs, mta, rl, wn);
            o_rl = o;
            wlim_n = win_lim(mta);
            if constexpr (!CHO) {
                if (lane == chunk.l && ((mta ^ m0) & (1u << 20)) == 0u) {
                    int i2, pg2, c2;
                    mt_unpack(mta, i2, pg2, c2);
                    mta = mt_pack(i2, chunk_pg, c2);
                }
            }
            stamp(4);
        }
        wg_barrier();
        if constexpr (CHO) {  // the output wave's last chunks (stored and published before the barrier)
            const uint32_t v = sm.cpg[lane];
            int ia, pga, ca;
            mt_unpack(mta, ia, pga, ca);
            if ((v >> 31) && (int)((v >> 10) & 1u) == ca && (int)(v & 0x3FFu) > pga)
                mta = mt_pack(ia, (int)(v & 0x3FFu), ca);
        }
        // the committed word's next-generation progress: mta's where both are
        // in one generation, else complete (mta's generation is mtc's next)
        {
            int ic, pgc, cc, ia, pga, ca;
            mt_unpack(mtc, ic, pgc, cc);
            mt_unpack(mta, ia, pga, ca);
            mtc = mt_keep(mtc, mt_pack(ic, cc == ca ? pga : kMtN, cc));
        }
#pragma unroll
        // the spawned pieces' counts = cq less the queue head's, which cq
        // already holds (cq = cnt_r + the head's count throughout the loop)
        for (int i = 0; i < 7; ++i) ss(ST_STAT_COUNT0 + i) = (uint32_t)(cq[i] - (i == q0 ? 1 : 0));
        ss(ST_STAT_MT_INDEX) = mtc;
        wave_sync();
    } else {
        // ================================================================ output
        const bool wide_obs = (p.n & 3) == 0 && e0 + kWave <= p.n && (reinterpret_cast<uintptr_t>(p.obs) & 15u) == 0;
        // packed obs: this wave builds the next-generation chunks (it idles
        // most of each step), one per two steps, for the lowest lane the draw
        // wave's cw word names; the new progress is published (cpg) right
        // after the chunk's stores are issued, and the wave's own last chunk
        // overrides a cw that does not show it yet.  A draw reads words past
        // index 623 only once the whole successor is published, 9+ chunks
        // after next[0..15] were stored (and each later chunk's operand
        // loads waited for those stores: one in-order vmcnt); the draw wave's
        // cooperative finish (mt_finish) rebuilds a successor from word 0,
        // not trusting the progress (MT words are deterministic: a chunk
        // racing it writes the same values).
        [[maybe_unused]] const MtRes orm = mt_res(p.mt + e0 * kMtPitch, lane);
        [[maybe_unused]] int last_l = -1, last_cur = 0, last_pg = 0;
        // a chunk's operands are issued at the end of a step and its words
        // computed and stored after the next step's obs stores: the loads have
        // a whole step to arrive, and the obs of a step never waits for them
        // (one in-order vmcnt: the wait covers only what was issued before)
        [[maybe_unused]] MtChunk ch;
        ch.l = -1;
        auto chunk_next = [&]() {
            const uint32_t w = sm.cw[lane];
            int pg = (int)(w & 0x3FFu);
            const int cur = (int)((w >> 10) & 1u);
            if (lane == last_l && cur == last_cur && last_pg > pg) pg = last_pg;
            mt_chunk_issue_pc(orm, (w >> 31) != 0u && pg < kMtN, pg, cur, lane, ch);
        };
        auto chunk_done = [&]() {
            const int npg = mt_chunk_store<0>(orm, lane, ch);
            if (ch.l >= 0) {
                last_l = ch.l;
                last_cur = ch.cur;
                last_pg = npg;
                if (lane == last_l) sm.cpg[lane] = 0x80000000u | ((uint32_t)last_cur << 10) | (uint32_t)last_pg;
            }
        };
        // one loop per obs mode (wave-uniform for the launch): the mode fixes
        // the number of obs stores per step, so the compiler's vmcnt for the
        // previous step's chunk operands counts exactly (with a runtime
        // branch it took the smallest count over the paths and waited for
        // the obs stores too)
        auto out_loop = [&](auto om_c) {
            constexpr int OM = decltype(om_c)::value;  // 0: no packed obs, 1: 16-B rows, 2: one dword per row
            // (WT: the 16-B row groups read once per lane, compile-time rows)
            constexpr bool EARLY = OM == 1 && !F32 && WT != 0;
            auto step_out = [&](int t, auto dn_c, auto nx_c) {
                lds_flag_wait_ge(&sm.fo, (uint32_t)t + 1u);
                stamp(1);
                uint32_t *const obs_t = p.obs ? p.obs + (int64_t)t * W * p.n : nullptr;
                if constexpr (OM != 0) {
                    if constexpr (EARLY) {
                        // read the planes, clear the overlay, raise fq, THEN
                        // store: the logic wave waits for fq before it changes
                        // a plane, and only the reads have to precede that
                        // (timing ablation: that wait cost the logic ~2%)
                        const auto ro = buf_rsrc(obs_t, (uint32_t)W * (uint32_t)p.n * 4u);
                        const uint32_t noff = (uint32_t)lrow * (uint32_t)p.n + (uint32_t)lcc;
                        uint4 ob[NBQ];
    #pragma unroll
                        for (int q = 0; q < NBQ; ++q) {
                            const int i = (4 * q + lrow + kPad) * kWave + lcc;
                            const uint4 v = *reinterpret_cast<const uint4 *>(&L[i]);
                            const uint4 o = *reinterpret_cast<const uint4 *>(&OV[i]);
                            ob[q] = make_uint4((v.x | o.x) & hmask, (v.y | o.y) & hmask, (v.z | o.z) & hmask,
                                               (v.w | o.w) & hmask);
                        }
    #pragma unroll
                        for (int q = 0; q < NBQ; ++q)  // (each lane clears the slots it read)
                            if (4 * q + lrow < W)
                                *reinterpret_cast<uint4 *>(&OV[(4 * q + lrow + kPad) * kWave + lcc]) =
                                    make_uint4(0u, 0u, 0u, 0u);
                        if (lane == 0) lds_flag_set(&sm.fq, (uint32_t)t + 1u);  // the logic wave may change the planes
    #pragma unroll
                        for (int q = 0; q < NBQ; ++q)
                            buf_store16<kNT>(ro,
                                             4 * q + lrow < W
                                                 ? ((uint32_t)e0 + (uint32_t)(4 * q) * (uint32_t)p.n + noff) * 4u
                                                 : kOff,
                                             ob[q]);
                    } else if constexpr (OM == 1) {
                        const auto ro = buf_rsrc(obs_t, (uint32_t)W * (uint32_t)p.n * 4u);
                        const uint32_t noff = (uint32_t)lrow * (uint32_t)p.n + (uint32_t)lcc;
    #pragma unroll
                        for (int q = 0; q < NBQ; ++q) {
                            if (WT || 4 * q < W) {
                                // rows past W (the last group's spare lanes) read
                                // the wall columns and store with an out-of-range
                                // offset: no branch around the store, so every
                                // step issues the same stores (exact vmcnt counts)
                                const bool on = 4 * q + lrow < W;
                                const int i = (4 * q + lrow + kPad) * kWave + lcc;
                                uint4 v = *reinterpret_cast<const uint4 *>(&L[i]);
                                const uint4 o = *reinterpret_cast<const uint4 *>(&OV[i]);
                                v.x = (v.x | o.x) & hmask;
                                v.y = (v.y | o.y) & hmask;
                                v.z = (v.z | o.z) & hmask;
                                v.w = (v.w | o.w) & hmask;
                                buf_store16<kNT>(
                                    ro, on ? ((uint32_t)e0 + (uint32_t)(4 * q) * (uint32_t)p.n + noff) * 4u : kOff, v);
                            }
                        }
                    } else if (real) {  // ragged / unaligned: one dword per row (rare: not tuned)
                        const auto ro = buf_rsrc(obs_t, (uint32_t)W * (uint32_t)p.n * 4u);
    #pragma unroll 1
                        for (int x = 0; x < W; ++x)
                            __builtin_amdgcn_raw_buffer_store_b32((col(L, x) | col(OV, x)) & hmask, ro,
                                                                  ((uint32_t)x * (uint32_t)p.n + (uint32_t)e) * 4u, 0, kNT);
                    }
                }
                if constexpr (F32) {
                    // float32 obs [n][W][H] of the wave's envs: one contiguous block,
                    // lane-consecutive float4 chunks, non-temporal (A/B: -13% f32 rollout)
                    const int64_t nreal64 = p.n - e0 < kWave ? p.n - e0 : kWave;
                    const int nreal = (int)nreal64;
                    float *out = p.obs_f32 + ((int64_t)t * p.n + e0) * (W * H);
                    if constexpr (WT != 0 && HT % 4 == 0) {
                        constexpr int CPC = HT / 4, CPE = WT * CPC;
                        uint32_t *O = sm.O;
    #pragma unroll
                        for (int x = 0; x < WT; ++x) O[lane * (WT + 1) + x] = (col(L, x) | col(OV, x)) & hmask;
                        wave_sync();
                        float4 *out4 = reinterpret_cast<float4 *>(out);
                        const float4 *F4 = reinterpret_cast<const float4 *>(sm.F4);
                        const int total = nreal * CPE;
                        for (int c = lane; c < total; c += kWave) {
                            const int ee = c / CPE;
                            const int cr = c - ee * CPE;
                            const int x = cr / CPC;
                            const int q = cr - x * CPC;
                            const float4 f = F4[(O[ee * (WT + 1) + x] >> (4 * q)) & 15u];
                            typedef float f32x4 __attribute__((ext_vector_type(4)));
                            const f32x4 fv = {f.x, f.y, f.z, f.w};
                            __builtin_nontemporal_store(fv, reinterpret_cast<f32x4 *>(&out4[c]));
                        }
                        wave_sync();  // staging reads done before the next step's writes
                    } else {
                        const int per_env = W * H;
                        const int total = nreal * per_env;
                        for (int f = lane; f < total; f += kWave) {
                            const int ee = f / per_env;
                            const int rem = f - ee * per_env;
                            const int x = rem / H;
                            const int y = rem - x * H;
                            const uint32_t w = (L[(x + kPad) * kWave + ee] | OV[(x + kPad) * kWave + ee]) & hmask;
                            out[f] = (float)((w >> y) & 1u);
                        }
                    }
                }
                stamp(3);
                if constexpr (!EARLY) {
                    wave_sync();  // every read of the overlay plane precedes its clearing
    #pragma unroll
                    for (int q = 0; q < NBQ; ++q)
                        if ((WT || 4 * q < W) && 4 * q + lrow < W)
                            *reinterpret_cast<uint4 *>(&OV[(4 * q + lrow + kPad) * kWave + lcc]) =
                                make_uint4(0u, 0u, 0u, 0u);
                }
                {
                    // reward / done of step t (and a reset's episode counters): branch-free
                    // stores, out-of-range offsets where there is nothing to store
                    const auto rr = buf_rsrc(p.reward ? p.reward + (int64_t)t * p.n : nullptr, (uint32_t)p.n * 4u);
                    const auto rd = buf_rsrc(p.done ? p.done + (int64_t)t * p.n : nullptr, (uint32_t)p.n);
                    const uint32_t dn = sm.dn[t & 1][lane];
                    if (!(kAblate & 64u)) {
                        __builtin_amdgcn_raw_buffer_store_b32(sm.rw[t & 1][lane], rr, real ? (uint32_t)e * 4u : kOff, 0, kRD);
                        __builtin_amdgcn_raw_buffer_store_b8((char)dn, rd, real ? (uint32_t)e : kOff, 0, kRD);
                        const bool rs_now = dn != 0u && p.autoreset == ST_AUTORESET_SAME_STEP;
                        const auto rs = buf_rsrc(p.stats, (uint32_t)ST_NSTAT * (uint32_t)sd * 4u);
                        const uint32_t eo = (uint32_t)e * 4u;
                        constexpr int kEpRow[4] = {ST_STAT_EP_TIME, ST_STAT_EP_SCORE, ST_STAT_EP_LINES, ST_STAT_EP_HOLES};
#pragma unroll
                        for (int k = 0; k < 4; ++k)
                            __builtin_amdgcn_raw_buffer_store_b32(sm.ep[t & 1][k][lane], rs,
                                                                  rs_now ? eo + (uint32_t)kEpRow[k] * (uint32_t)sd * 4u : kOff, 0, kST);
                    }
                }
                if constexpr (!EARLY)
                    if (lane == 0) lds_flag_set(&sm.fq, (uint32_t)t + 1u);  // the logic wave may change the planes
                stamp(4);
                if constexpr (CHO) {
                    if constexpr (decltype(dn_c)::value) chunk_done();  // the previous chunk (none at first: ch.l < 0)
                    stamp(5);
                    if constexpr (decltype(nx_c)::value) chunk_next();
                }
                stamp(2);
            };
            if constexpr (CHO) {
                // one chunk per two steps -- issued at even steps, computed
                // and stored at odd ones (the unrolled pair keeps every vmcnt
                // exact): 32 words per step and wave against the ~19 its 64
                // envs' draws consume (p_lock 0.21 x ~1.4 words per draw);
                // a chunk every step left the output wave's stores the
                // step's bottleneck (round 5: 1.268 -> 1.24 us per step,
                // profiles/r05/ab_rollout_chunk_every_other_step.txt)
                for (int t = 0; t < K; t += 2) {
                    step_out(t, std::false_type{}, std::true_type{});
                    if (t + 1 < K) step_out(t + 1, std::true_type{}, std::false_type{});
                }
            } else {
                for (int t = 0; t < K; ++t) step_out(t, std::true_type{}, std::true_type{});
            }
        };
        if (!p.obs || (kAblate & 8u)) out_loop(std::integral_constant<int, 0>{});
        else if (wide_obs) out_loop(std::integral_constant<int, 1>{});
        else out_loop(std::integral_constant<int, 2>{});
        if constexpr (CHO) chunk_done();
        wg_barrier();
    }
    // ---- counter rows this wave owns (logic: 0-5 and the piece row, draw:
    // the shape counts and the MT word) ----
    if constexpr (ROLE != kRoleO) {
        constexpr uint32_t kRowsD = ((1u << 7) - 1u) << ST_STAT_COUNT0 | 1u << ST_STAT_MT_INDEX;
        constexpr uint32_t kOwn = ROLE == kRoleD ? kRowsD : ((1u << kHotRows) - 1u) & ~kRowsD;
        const auto rs = buf_rsrc(p.stats, (uint32_t)kHotRows * (uint32_t)sd * 4u);
        const uint32_t soff = (uint32_t)e0 * 4u + loff * 4u;
#pragma unroll
        for (int q = 0; q < kHotQ; ++q) {
            if (((kOwn >> (4 * q)) & 0xFu) == 0u) continue;
            const bool st = (kOwn >> (4 * q + lrow)) & 1u;
            buf_store16<kST>(rs, st ? soff + (uint32_t)(4 * q) * (uint32_t)sd * 4u : kOff,
                             *reinterpret_cast<const uint4 *>(&SS[(4 * q + lrow) * kWave + lcc]));
        }
    }
    if constexpr (STAMP) {
        uint64_t *slot = p.stamps + (int64_t)blockIdx.x * kStampWords + 16 * (ROLE == kRoleL ? 0 : ROLE == kRoleD ? 1 : 2);
        if (lane == 0) {
#pragma unroll
            for (int i = 0; i < 12; ++i) slot[i] = tacc[i];
            slot[12] = __builtin_amdgcn_s_memrealtime() - rt0;
            slot[13] = (uint64_t)K;
        }
    }
}

// (Capping it at 85 VGPRs -- six waves per SIMD, so 131,072 envs fit at once
// -- spills and loses at 65,536 envs: 1.72 -> 2.08 us per step; launch_rollout
// runs the two-wave rollout above 4 workgroups per CU instead.)
template <int WT, int HT, bool F32, bool SC0 = false, bool STAMP = false>
__global__ __launch_bounds__(3 * kWave) void k_rollout(KParams p) {
    __shared__ RoLds<WT, F32> sm;
    if (threadIdx.x < kWave) rollout_wave<WT, HT, F32, SC0, STAMP, kRoleL>(p, sm);
    else if (threadIdx.x < 2 * kWave) rollout_wave<WT, HT, F32, SC0, STAMP, kRoleD>(p, sm);
    else rollout_wave<WT, HT, F32, SC0, STAMP, kRoleO>(p, sm);
}

// The two-wave rollout (run_steps, board and counters in LDS): launch_rollout
// takes it for batches of more than 4 workgroups per CU, where the three-wave
// kernel's extra waves and window reloads cost more than its shorter logic
// chain gains (131,072 envs: 2.8 against 4.0 us per step).
template <int WT, int HT, bool F32, bool SC0 = false>
__global__ __launch_bounds__(2 * kWave) void k_rollout2(KParams p) {
    __shared__ StepLds<WT, F32, 0> sm;
    if (threadIdx.x < kWave) run_steps<WT, HT, F32, false, 0, SC0, kRoleL>(p, sm);
    else run_steps<WT, HT, F32, false, 0, SC0, kRoleD>(p, sm);
}

// no scoring flags (SC0 specializations of the 10x20 kernels)
constexpr uint32_t kScoringFlags =
    ST_PENALISE_HEIGHT | ST_PENALISE_HEIGHT_INCREASE | ST_ADVANCED_CLEARS | ST_HIGH_SCORING |
    ST_PENALISE_HOLES | ST_PENALISE_HOLES_INCREASE;

// ---------------------------------------------------------------- reset
// TetrisEngine.clear (tetris_env.py:306-315) on masked envs.  n_deaths,
// shape_counts and the lock-delay counter persist (R15).
__global__ __launch_bounds__(kWave) void k_reset(KParams p) {
    __shared__ uint32_t S[kMtN];
    const int lane = threadIdx.x;
    const int64_t e0 = (int64_t)blockIdx.x * kWave;
    const int64_t e = e0 + lane;
    const int64_t sd = p.stride;
    const bool m = e < p.n && (p.mask == nullptr || p.mask[e] != 0);
    int32_t *st = p.stats + e;
    int32_t cnt[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) cnt[i] = st[(ST_STAT_COUNT0 + i) * sd];
    uint32_t mtst = (uint32_t)st[ST_STAT_MT_INDEX * sd];
    const uint32_t mt0 = mtst;
    const uint32_t pw = p.piece[e];
    const MtPre nopre{};
    // the new piece: the preview, or (none valid) a draw; then the next preview
    int sid = pv_id(mt0);
    const bool need1 = m && !pv_ok(mt0);
    if (__ballot(need1)) {
        const int pk = draw_shape<8, false>(need1, cnt, mtst, p.mt + e0 * kMtPitch, S, lane, nopre, false);
        if (need1) sid = pk;
    }
#pragma unroll
    for (int i = 0; i < 7; ++i) cnt[i] += (m && i == sid);  // _new_piece :199
    const uint32_t m1 = mtst;
    const int npv = draw_shape<8, false>(m, cnt, mtst, p.mt + e0 * kMtPitch, S, lane, nopre, false);
    if (m) {
        st[ST_STAT_TIME * sd] = 0;
        st[ST_STAT_SCORE * sd] = 0;
        st[ST_STAT_HOLES * sd] = 0;
        st[ST_STAT_LINES * sd] = 0;
        st[ST_STAT_PIECE_HEIGHT * sd] = 0;
        st[ST_STAT_MT_INDEX * sd] = (int32_t)pv_pack(mtst, npv, mt_consumed(m1, mtst));
#pragma unroll
        for (int i = 0; i < 7; ++i) st[(ST_STAT_COUNT0 + i) * sd] = cnt[i];
        for (int x = 0; x < p.W; ++x) p.board[x * sd + e] = 0u;
        p.piece[e] = pack_piece(sid, 0, p.W / 2, 0, (int)(pw >> 17));
    }
}

// ---------------------------------------------------------------- seed
// random.seed(s): init_by_array(key = 32-bit limbs of s) (+ the first twist
// into the second buffer), and the counter values of TetrisEngine.__init__
// (:165-181).  One lane per env, serial (one-time).
__global__ void k_seed(KParams p) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= p.stride) return;
    const uint64_t s = p.seeds[e];
    const uint32_t key[2] = {(uint32_t)s, (uint32_t)(s >> 32)};
    const int len = (s >> 32) ? 2 : 1;
    uint32_t *g = p.mt + e * kMtPitch;  // buffer A
    uint32_t prev = 19650218u;  // init_genrand(19650218)
    g[0] = prev;
    for (int i = 1; i < kMtN; ++i) {
        prev = 1812433253u * (prev ^ (prev >> 30)) + (uint32_t)i;
        g[i] = prev;
    }
    int i = 1, j = 0;
    prev = g[0];
    for (int k = kMtN > len ? kMtN : len; k; --k) {
        const uint32_t v = (g[i] ^ ((prev ^ (prev >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
        g[i] = v;
        prev = v;
        ++i;
        ++j;
        if (i >= kMtN) {
            g[0] = g[kMtN - 1];
            i = 1;
        }
        if (j >= len) j = 0;
    }
    for (int k = kMtN - 1; k; --k) {
        const uint32_t v = (g[i] ^ ((prev ^ (prev >> 30)) * 1566083941u)) - (uint32_t)i;
        g[i] = v;
        prev = v;
        ++i;
        if (i >= kMtN) {
            g[0] = g[kMtN - 1];
            i = 1;
        }
    }
    g[0] = 0x80000000u;
    // A now holds CPython's state after random.seed (index 624: the first
    // draw twists).  The first twist goes to B as the complete next
    // generation (genrand_uint32 with index == N, out of place), so the
    // first draw switches to it like any other generation end, and
    // st_mt_sync of a fresh context returns exactly random.getstate().
    uint32_t *nx = g + kMtB;
    int kk = 0;
    for (; kk < kMtN - 397; ++kk) nx[kk] = g[kk + 397] ^ mt_mix(g[kk], g[kk + 1]);
    for (; kk < kMtN - 1; ++kk) nx[kk] = nx[kk + (397 - kMtN)] ^ mt_mix(g[kk], g[kk + 1]);
    nx[kMtN - 1] = nx[396] ^ mt_mix(g[kMtN - 1], nx[0]);

    const int64_t sd = p.stride;
    int32_t *st = p.stats + e;
    for (int r = 0; r < ST_NSTAT; ++r) st[r * sd] = 0;
    st[ST_STAT_TIME * sd] = -1;   // :165
    st[ST_STAT_SCORE * sd] = -1;  // :166
    st[ST_STAT_MT_INDEX * sd] = (int32_t)mt_pack(kMtN, kMtN, 0);  // index 624, next generation complete
    for (int x = 0; x < p.W; ++x) p.board[x * sd + e] = 0u;
    p.piece[e] = pack_piece(0, 0, p.W / 2, 0, 0);
}

// ---------------------------------------------------------------- MT sync
// st_mt_sync: every env back to CPython's form (see "Double-buffered twist"):
// the preview's words are given back (the reference has not drawn it: its
// state is c words earlier, in the previous generation if the preview's draw
// crossed index 624 -- that buffer is intact, no next-generation block has
// been built since the switch), the generation holding that position is
// copied to A if it is B, and the index loses the engine bits (the next
// generation's progress restarts at 0, the preview is dropped: the next spawn
// draws its piece, then a new preview).  One wave per 64 envs; it copies its
// lanes' B buffers one env at a time, cooperatively.
__global__ __launch_bounds__(kWave) void k_mt_sync(KParams p) {
    const int lane = threadIdx.x;
    const int64_t e0 = (int64_t)blockIdx.x * kWave;
    const int64_t e = e0 + lane;
    int32_t *row = p.stats + (int64_t)ST_STAT_MT_INDEX * p.stride;
    const uint32_t r = (uint32_t)row[e];
    int idx = (int)(r & 0x3FFu);
    uint32_t cur = (r >> 20) & 1u;
    if (pv_ok(r)) {
        // A preview draw always starts where an earlier draw ended (index
        // >= 1 of its generation), so idx > c: it stayed in one generation;
        // idx <= c: it started at index 624 - (c - idx) of the previous one,
        // which is intact (nothing is built into it while the preview is
        // pending).  idx == c is a draw that started exactly at 624: CPython
        // holds the old words with index 624 (it twists lazily).
        const int c = (int)((r >> 25) & kPvCMax);
        if (idx > c) {
            idx -= c;
        } else {
            idx = kMtN - (c - idx);
            cur ^= 1u;
        }
    }
    uint64_t inb = __ballot(cur);
    while (inb) {
        const int l = __builtin_ctzll(inb);
        inb &= inb - 1;
        uint32_t *g = p.mt + (e0 + l) * kMtPitch;
        uint32_t t[10];
#pragma unroll
        for (int q = 0; q < 10; ++q) {
            const int i = lane + kWave * q;
            t[q] = i < kMtN ? g[kMtB + i] : 0u;
        }
#pragma unroll
        for (int q = 0; q < 10; ++q) {
            const int i = lane + kWave * q;
            if (i < kMtN) g[i] = t[q];
        }
    }
    if (r != (uint32_t)idx) row[e] = idx;
}

// ---------------------------------------------------------------- render
// TetrisEngine.render() (tetris_env.py:317-321): board + current piece.
__global__ __launch_bounds__(kWave) void k_render(KParams p) {
    __shared__ uint32_t L[(kMaxW + 2 * kPad) * kWave];
    const int lane = threadIdx.x;
    const int64_t e = (int64_t)blockIdx.x * kWave + lane;
    const int64_t sd = p.stride;
    const int W = p.W;
    const uint32_t hmask = (1u << p.H) - 1u;
    for (int x = 0; x < W; ++x) lcol(L, x, lane) = p.board[x * sd + e];
    for (int x = 0; x < kPad; ++x) {
        L[x * kWave + lane] = 0u;
        L[(W + kPad + x) * kWave + lane] = 0u;
    }
    const uint32_t pw = p.piece[e];
    const uint32_t t = (pw & 7u) * 4 + ((pw >> 3) & 3u);
    paint(L, lane, c_tab_m[t], c_tab_g[t], (int)((pw >> 5) & 63u), (int)((pw >> 11) & 63u), hmask);
    if (e < p.n)
        for (int x = 0; x < W; ++x) p.obs[x * p.n + e] = lcol(L, x, lane) & hmask;
}

// ---------------------------------------------------------------- export
// st_export_env: one env's outputs and state as one record (the single-env
// surface's per-step read-back in one transfer): obs words | reward | done |
// stats rows | MT words (optional) | float32 obs (optional).  The MT index
// row and words are CPython's form, computed read-only the way k_mt_sync
// rewrites them (the preview's words given back, the generation holding that
// position): the env keeps its preview and next-generation progress.  The
// float32 obs saves the host the bit unpacking (the record is written
// straight into mapped pinned memory).
__global__ __launch_bounds__(256) void k_export(KParams p, int64_t env, const uint32_t *obs,
                                               const int32_t *rew, const uint8_t *done, uint32_t parts,
                                               uint32_t *out) {
    const int W = p.W, H = p.H;
    const int head = W + 2 + ST_NSTAT;
    const uint32_t r = (uint32_t)p.stats[(int64_t)ST_STAT_MT_INDEX * p.stride + env];
    int idx = (int)(r & 0x3FFu);
    uint32_t cur = (r >> 20) & 1u;
    if (pv_ok(r)) {  // see k_mt_sync
        const int c = (int)((r >> 25) & kPvCMax);
        if (idx > c) {
            idx -= c;
        } else {
            idx = kMtN - (c - idx);
            cur ^= 1u;
        }
    }
    for (int i = threadIdx.x; i < head; i += blockDim.x) {
        uint32_t v;
        if (i < W) v = obs ? obs[(int64_t)i * p.n + env] : 0u;
        else if (i == W) v = rew ? (uint32_t)rew[env] : 0u;
        else if (i == W + 1) v = done ? (uint32_t)done[env] : 0u;
        else if (i == W + 2 + ST_STAT_MT_INDEX) v = (uint32_t)idx;
        else v = (uint32_t)p.stats[(int64_t)(i - W - 2) * p.stride + env];
        out[i] = v;
    }
    if (parts & ST_EXPORT_MT) {
        const uint32_t *g = p.mt + env * kMtPitch + (cur ? kMtB : 0u);
        for (int i = threadIdx.x; i < kMtN; i += blockDim.x) out[head + i] = g[i];
    }
    if (parts & ST_EXPORT_OBS_F32) {
        float *f = reinterpret_cast<float *>(out + head + kMtN);
        for (int i = threadIdx.x; i < W * H; i += blockDim.x) {
            const int x = i / H, y = i - x * H;
            const uint32_t w = obs ? obs[(int64_t)x * p.n + env] : 0u;
            f[i] = (float)((w >> y) & 1u);
        }
    }
}

// ---------------------------------------------------------------- misc
// Image writers: the output of a block of envs is one contiguous region, so
// lanes walk it in 16-B chunks (lane-consecutive vector stores, one 1-KB
// burst per wave instruction, non-temporal: the images stream past L2), and
// each chunk's elements are decoded from the block's packed obs words staged
// in LDS.  Reads are 4 B per env per board column, coalesced over the
// block's envs.
// 2 envs per block: the blocks' regions are 2 x 28 KB (grayscale 84 f32), so
// the concurrently written regions sit closer together than with 16 envs
// (tools/ab_img.py at 65,536 envs: 84 gray f32 386 -> 356 us, 160 rgb u8
// 2,350 -> 2,072 us; tools/write_bw.hip shows the same effect on bare stores)
constexpr int kImgEnvs = 2;  // envs per block
constexpr int kMaxImg = 4096;  // largest image side (st_grayscale checks)

template <typename T>
__device__ __forceinline__ void store16_nt(T *dst, const T (&v)[16 / sizeof(T)]) {
    typedef unsigned int u4 __attribute__((ext_vector_type(4)));
    u4 w;
    __builtin_memcpy(&w, v, 16);
    __builtin_nontemporal_store(w, reinterpret_cast<u4 *>(dst));
}

// packed obs [W][n] -> float32 [n][W][H] (TetrisEnv.step float32 cast, :400):
// 64 envs per block, element (e, x, y) = bit y of word (x, e).
__global__ __launch_bounds__(256) void k_obs_f32(const uint32_t *__restrict__ obs, float *__restrict__ out,
                                                 int64_t n, int W, int H) {
    __shared__ uint32_t O[kWave * kMaxW];
    const int64_t e0 = (int64_t)blockIdx.x * kWave;
    const int ne = (int)(n - e0 < kWave ? n - e0 : kWave);
    for (int i = threadIdx.x; i < W * kWave; i += blockDim.x) {
        const int x = i / kWave, l = i - x * kWave;
        if (l < ne) O[l * W + x] = obs[(int64_t)x * n + e0 + l];
    }
    __syncthreads();
    const int per = W * H;
    const int total = ne * per;  // elements of this block's contiguous region
    float *base = out + e0 * per;
    if ((reinterpret_cast<uintptr_t>(base) & 15u) == 0 && (total & 3) == 0) {
        for (int c = threadIdx.x; 4 * c < total; c += blockDim.x) {
            int f = 4 * c;
            int le = f / per, rem = f - le * per;
            int x = rem / H, y = rem - x * H;
            float v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                v[j] = (float)((O[le * W + x] >> y) & 1u);
                if (++y == H) {
                    y = 0;
                    if (++x == W) {
                        x = 0;
                        ++le;
                    }
                }
            }
            store16_nt(base + f, v);
        }
    } else {
        for (int f = threadIdx.x; f < total; f += blockDim.x) {
            const int le = f / per, rem = f - le * per;
            const int x = rem / H, y = rem - x * H;
            base[f] = (float)((O[le * W + x] >> y) & 1u);
        }
    }
}

// convert_grayscale (tetris_env.py:76-114) [+ the rgb channel repeat, :117-122]
// in closed form.  The reference transposes the (W, H) board to (H, W),
// scales each cell to blk x blk, puts `gap` background lines before every
// block row/column and after the last, then centres the result with border
// (0) padding.  Image row r maps to board row y, column c to board column x;
// the two maps (-2 border, -1 background line, else the board index) are
// tabulated in LDS once per block, so a pixel is two table reads and a bit
// test: 0 (border), 128 (background), 190 (cell).
template <typename T, int CH>
__global__ __launch_bounds__(256) void k_grayscale(const uint32_t *__restrict__ obs, T *__restrict__ out,
                                                   int64_t n, int W, int H, int size) {
    constexpr int channels = CH;
    __shared__ uint32_t O[kImgEnvs * kMaxW];
    __shared__ int8_t RM[kMaxImg], CM[kMaxImg];
    const int64_t e0 = (int64_t)blockIdx.x * kImgEnvs;
    const int ne = (int)(n - e0 < kImgEnvs ? n - e0 : kImgEnvs);
    const int lim = W > H ? W : H;
    const int gap = size / 100 + 1;
    const int blk = (size - 2 * gap) / lim - gap;
    const int pitch = blk + gap;
    const int pr = (size - (gap + pitch * H)) / 2;  // padding_width  (axis 0 = y)
    const int pc = (size - (gap + pitch * W)) / 2;  // padding_height (axis 1 = x)
    for (int i = threadIdx.x; i < size; i += blockDim.x) {
        const int r = i - pr, c = i - pc;
        RM[i] = (int8_t)((r < 0 || r >= gap + pitch * H) ? -2 : (r % pitch < gap ? -1 : r / pitch));
        CM[i] = (int8_t)((c < 0 || c >= gap + pitch * W) ? -2 : (c % pitch < gap ? -1 : c / pitch));
    }
    for (int i = threadIdx.x; i < W * kImgEnvs; i += blockDim.x) {
        const int x = i / kImgEnvs, l = i - x * kImgEnvs;
        if (l < ne) O[l * kMaxW + x] = obs[(int64_t)x * n + e0 + l];
    }
    __syncthreads();
    const int per = size * size * channels;  // elements per env
    const int total = ne * per;
    T *base = out + e0 * per;
    auto pix = [&](int le, int r, int c) -> T {
        const int y = RM[r], x = CM[c];
        const uint32_t v = (y == -2 || x == -2) ? 0u
                           : (y < 0 || x < 0) ? 128u
                           : (((O[le * kMaxW + x] >> y) & 1u) ? 190u : 128u);
        return (T)v;
    };
    // A thread writes one 16-B chunk per iteration, lane-consecutive (48-B
    // lane strides -- a thread taking an rgb period of 3 chunks -- measured 5x
    // slower).  Gray (CH == 1): a chunk is V whole pixels, each decoded once.
    // RGB: the chunk's elements are decoded one by one (decoding only where a
    // new pixel starts measured slower: divergent LDS reads).  The position
    // advances by the block's stride through block-uniform digits: no
    // runtime division in the loop.
    constexpr int V = 16 / (int)sizeof(T);  // elements per chunk
    if ((reinterpret_cast<uintptr_t>(base) & 15u) == 0 && (total % V) == 0) {
        const int S = (int)blockDim.x * V;  // elements per block iteration
        const int sk = S % channels, sp = S / channels;
        const int sc = sp % size, sr = (sp / size) % size, sl = sp / (size * size);
        int f = V * (int)threadIdx.x;
        int le = f / per, rem = f - le * per;
        int pp = rem / channels, k = rem - pp * channels;
        int r = pp / size, c = pp - r * size;
        for (; f < total; f += S) {
            T v[V];
            int jk = k, jc = c, jr = r, jl = le;
#pragma unroll
            for (int j = 0; j < V; ++j) {
                v[j] = pix(jl, jr, jc);
                if (CH == 1 || ++jk == channels) {
                    jk = 0;
                    if (++jc == size) {
                        jc = 0;
                        if (++jr == size) {
                            jr = 0;
                            ++jl;
                        }
                    }
                }
            }
            store16_nt(base + f, v);
            k += sk;
            if (k >= channels) {
                k -= channels;
                ++c;
            }
            c += sc;
            if (c >= size) {
                c -= size;
                ++r;
            }
            r += sr;
            if (r >= size) {
                r -= size;
                ++le;
            }
            le += sl;
        }
    } else {
        for (int f = threadIdx.x; f < total; f += blockDim.x) {
            const int le = f / per, rem = f - le * per;
            const int p = rem / channels;
            base[f] = pix(le, p / size, p - (p / size) * size);
        }
    }
}

// The same images in sweep order: the grid strides over the WHOLE output, so
// that all waves write within one moving window of the image batch
// (tools/write_bw.hip: 16-B non-temporal store sweeps reach 5.8-6.0 TB/s with
// 128-1,024 workgroups, against 4.8-5.3 TB/s when every block owns a region
// of 16 .. 1 envs).  It pays for float32 rgb only: the per-element decode
// (two table reads and a lane shuffle) keeps the grayscale and u8 sweeps
// below the per-block kernel.  Per iteration a wave writes U
// consecutive 1-KB runs (64 lanes x 16 B); the U runs span at most two envs
// (64 V U <= size^2 CH, checked by the launcher), whose packed obs words the
// wave fetches once per iteration (one word per lane, the next iteration's
// prefetched under the current one's stores) and hands to each element with
// a lane shuffle.
constexpr int kImgSweepGrid = 1024;  // workgroups of the sweep (grid-stride)
constexpr int kImgRuns = 4;  // U: 1-KB runs per wave iteration
template <typename T, int CH>
__global__ __launch_bounds__(256) void k_grayscale_sweep(const uint32_t *__restrict__ obs, T *__restrict__ out,
                                                         int64_t n, int W, int H, int size) {
    __shared__ int8_t RM[kMaxImg], CM[kMaxImg];
    const int lim = W > H ? W : H;
    const int gap = size / 100 + 1;
    const int blk = (size - 2 * gap) / lim - gap;
    const int pitch = blk + gap;
    const int pr = (size - (gap + pitch * H)) / 2;
    const int pc = (size - (gap + pitch * W)) / 2;
    for (int i = threadIdx.x; i < size; i += blockDim.x) {
        const int r = i - pr, c = i - pc;
        RM[i] = (int8_t)((r < 0 || r >= gap + pitch * H) ? -2 : (r % pitch < gap ? -1 : r / pitch));
        CM[i] = (int8_t)((c < 0 || c >= gap + pitch * W) ? -2 : (c % pitch < gap ? -1 : c / pitch));
    }
    __syncthreads();
    constexpr int V = 16 / (int)sizeof(T);  // elements per 16-B chunk
    constexpr int U = kImgRuns;
    constexpr int RUN = kWave * V;  // elements per 1-KB run
    const int lane = threadIdx.x & (kWave - 1);
    const int per = size * size * CH;
    const int64_t total = n * (int64_t)per;
    // a position as (env, row, column, channel) digits, advanced by fixed
    // element counts without runtime division
    struct Pos {
        int64_t l;
        int r, c, k;
    };
    struct Step {
        int64_t l;
        int r, c, k;
    };
    auto mkstep = [&](int64_t d) -> Step {
        const int64_t l = d / per;
        const int q = (int)(d - l * per);
        const int p = q / CH;
        return Step{l, p / size, p % size, q - p * CH};
    };
    auto adv = [&](Pos x, const Step &d) -> Pos {
        x.k += d.k;
        if (x.k >= CH) {
            x.k -= CH;
            ++x.c;
        }
        x.c += d.c;
        if (x.c >= size) {
            x.c -= size;
            ++x.r;
        }
        x.r += d.r;
        if (x.r >= size) {
            x.r -= size;
            ++x.l;
        }
        x.l += d.l;
        return x;
    };
    const int64_t S = (int64_t)gridDim.x * (blockDim.x / kWave) * U * RUN;  // elements per grid iteration
    const Step dS = mkstep(S), dR = mkstep(RUN);
    const int64_t gw = (int64_t)blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave);
    int64_t f = gw * (U * RUN) + (int64_t)lane * V;
    Pos pos;
    {
        const Step s0 = mkstep(f);
        pos = Pos{s0.l, s0.r, s0.c, s0.k};
    }
    // this lane's word slot: env (lane / W) of the pair, column lane % W
    const int wx = lane % W, we = lane / W;
    const bool wlane = lane < 2 * W;
    auto fetch = [&](int64_t ea) -> uint32_t {
        const int64_t e = ea + we;
        return (wlane && e < n) ? obs[(int64_t)wx * n + e] : 0u;
    };
    auto first = [](int64_t v) -> int64_t {  // the wave's lowest-f active lane holds its lowest env
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
        const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
        return (int64_t)(((uint64_t)hi << 32) | lo);
    };
    int64_t ea = first(pos.l);
    uint32_t wcur = f < total ? fetch(ea) : 0u;
    for (; f < total; f += S) {
        const Pos nxt = adv(pos, dS);
        const bool more = f + S < total;
        const int64_t ean = first(more ? nxt.l : ea);
        const uint32_t wnext = more ? fetch(ean) : 0u;  // prefetch under this iteration's stores
        Pos q = pos;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t fu = f + (int64_t)u * RUN;
            if (fu < total) {
                T v[V];
                int jk = q.k, jc = q.c, jr = q.r;
                int64_t jl = q.l;
#pragma unroll
                for (int j = 0; j < V; ++j) {
                    const int y = RM[jr], x = CM[jc];
                    const int src = (int)(jl - ea) * W + (x < 0 ? 0 : x);
                    const uint32_t w = (uint32_t)__shfl((int)wcur, src);
                    const uint32_t px = (y == -2 || x == -2) ? 0u
                                        : (y < 0 || x < 0) ? 128u
                                        : (((w >> y) & 1u) ? 190u : 128u);
                    v[j] = (T)px;
                    if (CH == 1 || ++jk == CH) {
                        jk = 0;
                        if (++jc == size) {
                            jc = 0;
                            if (++jr == size) {
                                jr = 0;
                                ++jl;
                            }
                        }
                    }
                }
                store16_nt(out + fu, v);
            }
            if (u + 1 < U) q = adv(q, dR);
        }
        pos = nxt;
        ea = ean;
        wcur = wnext;
    }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void k_gen_actions(uint8_t *out, int64_t n, int64_t t, uint64_t seed, int64_t off) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    const uint64_t x = seed ^ (((uint64_t)t << 32) ^ (uint64_t)(off + e));
    out[e] = (uint8_t)(splitmix64(x) % 7ull);
}

// st_check_actions: a sticky flag for actions outside 0..6 (the reference's
// KeyError, tetris_env.py:245), 16 actions per lane from one 16-B load.  A
// byte b is > 6 iff b >= 0x80 or (b & 0x7F) + 0x79 reaches bit 7 (no carry
// leaves the byte).  Only lanes that saw one store the flag (vector stores).
__global__ __launch_bounds__(256) void k_check_actions(const uint8_t *__restrict__ a, int64_t n,
                                                       uint32_t *flag) {
    const int64_t i0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16;
    if (i0 >= n) return;
    bool bad = false;
    if (i0 + 16 <= n && (reinterpret_cast<uintptr_t>(a + i0) & 15u) == 0) {
        const uint4 v = *reinterpret_cast<const uint4 *>(a + i0);
        auto over6 = [](uint32_t w) { return ((((w & 0x7F7F7F7Fu) + 0x79797979u) | w) & 0x80808080u) != 0u; };
        bad = over6(v.x) || over6(v.y) || over6(v.z) || over6(v.w);
    } else {
        for (int64_t i = i0; i < n && i < i0 + 16; ++i) bad = bad || a[i] > 6;
    }
    if (bad) flag[0] = 1u;
}

// st_gate_actions: the same test over all n actions, reduced to one answer
// per call: words[0] = the gate the next step reads (the epoch if an action
// is outside 0..6, else 0), words[1] = blocks finished (the last one resets
// it), words[2] = the epoch once any block saw a bad action (epoch-tagged, so
// no word needs clearing between calls).  The last block publishes the gate
// and writes the host word -- epoch | bad << 31, system scope -- which
// st_gate_wait spins on: the host waits for this kernel alone.  Every
// atomic is a per-lane global atomic (no scalar-cache write).
__global__ __launch_bounds__(256) void k_gate_actions(const uint8_t *__restrict__ a, int64_t n, uint32_t *words,
                                                      uint32_t *host, uint32_t epoch) {
    auto over6 = [](uint32_t w) { return ((((w & 0x7F7F7F7Fu) + 0x79797979u) | w) & 0x80808080u) != 0u; };
    bool bad = false;
    const int64_t step = (int64_t)gridDim.x * blockDim.x * 16;
    for (int64_t i0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16; i0 < n; i0 += step) {
        if (i0 + 16 <= n && (reinterpret_cast<uintptr_t>(a + i0) & 15u) == 0) {
            const uint4 v = *reinterpret_cast<const uint4 *>(a + i0);
            bad = bad || over6(v.x) || over6(v.y) || over6(v.z) || over6(v.w);
        } else {
            for (int64_t i = i0; i < n && i < i0 + 16; ++i) bad = bad || a[i] > 6;
        }
    }
    // a wave that saw one tags words[2] and waits for the atomic's return, so
    // the tag is performed at L2 before its block counts itself done
    if (__ballot(bad) && (threadIdx.x & (kWave - 1)) == 0) {
        const uint32_t old = __hip_atomic_exchange(&words[2], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("" ::"v"(old));
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t done = __hip_atomic_fetch_add(&words[1], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (done == gridDim.x - 1) {  // the last block: every tag is in
            const bool any = __hip_atomic_load(&words[2], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == epoch;
            words[0] = any ? epoch : 0u;
            __hip_atomic_store(&words[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(host, epoch | (any ? 0x80000000u : 0u), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// ---------------------------------------------------------------- greedy policy
// Benchmark / test workload generator (not part of the reference env): the
// action a greedy placement player takes in every env's current state, so
// that rollouts clear lines (uniform random actions almost never do; SURVEY
// §8(d) asks for a clear-heavy variant).  For the current piece, every
// (rot 0..3, anchor x in [-3, W+3)) is hard-dropped from row 0 onto the
// board; score = 80*lines - 12*holes - 3*height - 2000*(piece above the top)
// (2 x the fixture generator's 40 / 6 / 1.5 / 1000, tests/golden/gen_golden.py
// greedy_target), first maximum in (rot, x) order.  The action turns the
// piece toward the target rotation (rotate_left), then moves it toward x,
// then hard-drops; with probability explore/1000 it is a uniform random
// action instead: splitmix64(seed ^ (t << 32 ^ e)).  Stateless: the target
// depends only on the board and the piece id.
__global__ __launch_bounds__(kWave) void k_policy_greedy(KParams p, uint64_t seed, int64_t t,
                                                         uint32_t explore, uint8_t *out) {
    constexpr int P = 8;  // wall columns each side: x + dx spans [-6, W + 5]
    __shared__ uint32_t L[(kMaxW + 2 * P) * kWave];
    const int lane = threadIdx.x;
    const int64_t e = (int64_t)blockIdx.x * kWave + lane;
    const int64_t sd = p.stride;
    const int W = p.W, H = p.H;
    const uint32_t hmask = (1u << H) - 1u, floorb = ~hmask;
    auto col = [&](int c) -> uint32_t & { return L[(c + P) * kWave + lane]; };
    for (int c = 0; c < W; ++c) col(c) = p.board[c * sd + e] | floorb;
    for (int c = 0; c < P; ++c) {
        col(c - P) = ~0u;
        col(W + c) = ~0u;
    }
    const uint32_t pw = p.piece[e];
    const int id = (int)(pw & 7u), rot = (int)((pw >> 3) & 3u), ax = (int)((pw >> 5) & 63u);
    int best_score = INT32_MIN, trot = -1, tx = 0;
    for (int r = 0; r < 4; ++r) {
        const uint32_t m = c_tab_m[id * 4 + r], g = c_tab_g[id * 4 + r];
        for (int x = -3; x < W + 3; ++x) {
            uint32_t v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = col(x + pc_dx(g, j));
            if (collides_v(m, 0, v)) continue;
            const int y = drop_v(g, 0, v);
            bool ok = true;
            uint32_t pb[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t byte = (m >> (8 * j)) & 0xFFu;
                ok = ok && y + __builtin_ctz(byte) - 3 >= 0;
                pb[j] = pc_bits(m, j, y) & hmask;
            }
            // the board with the piece: column c gets the bits of every
            // descriptor column at c (repeated last columns are idempotent)
            uint32_t andv = hmask;
            for (int c = 0; c < W; ++c) {
                uint32_t w = col(c);
#pragma unroll
                for (int j = 0; j < 4; ++j) w |= x + pc_dx(g, j) == c ? pb[j] : 0u;
                andv &= w;
            }
            const int lines = __builtin_popcount(andv);
            int holes = 0;
            uint32_t orv = 0;
            for (int c = 0; c < W; ++c) {
                uint32_t w = col(c);
#pragma unroll
                for (int j = 0; j < 4; ++j) w |= x + pc_dx(g, j) == c ? pb[j] : 0u;
                w = (andv ? compact(w & hmask, andv) : (w & hmask)) | floorb;
                holes += H - (int)__builtin_ctz(w) - __builtin_popcount(w & hmask);
                orv |= w & hmask;
            }
            const int height = orv ? H - (int)__builtin_ctz(orv) : 0;
            const int sc = 80 * lines - 12 * holes - 3 * height - (ok ? 0 : 2000);
            if (sc > best_score) {
                best_score = sc;
                trot = r;
                tx = x;
            }
        }
    }
    uint32_t a = 2u;  // no legal placement: hard drop
    if (trot >= 0) a = rot != trot ? 4u : (ax < tx ? 1u : (ax > tx ? 0u : 2u));
    const uint64_t h = splitmix64(seed ^ (((uint64_t)t << 32) ^ (uint64_t)e));
    if ((uint32_t)(h % 1000ull) < explore) a = (uint32_t)((h >> 32) % 7ull);
    if (e < p.n) out[e] = (uint8_t)a;
}

}  // namespace

hipError_t launch_seed(const KParams &p, hipStream_t s) {
    const int64_t blocks = (p.stride + 255) / 256;
    hipLaunchKernelGGL(k_seed, dim3((unsigned)blocks), dim3(256), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_reset(const KParams &p, hipStream_t s) {
    hipLaunchKernelGGL(k_reset, dim3((unsigned)(p.stride / kWave)), dim3(kWave), 0, s, p);
    return hipGetLastError();
}

// k_step's arguments: the preloaded six, then the whole KParams
#define ST_STEP_ARGS(p) (p).board, (p).stats, (p).actions, (p).mt, (p).stride, (p).n, (p)
hipError_t launch_step(const KParams &p, hipStream_t s) {
    const dim3 grid((unsigned)(p.stride / kWave)), block(2 * kWave);  // logic + draw wave
    const bool f32 = p.obs_f32 != nullptr;
    const bool sc0 = !(p.flags & kScoringFlags);
    if (p.final_obs || p.info || p.gate) {  // st_step_vec: the vector env's outputs (VEC); gated launches
        if (p.W == 10 && p.H == 20) {
            if (f32 && sc0) hipLaunchKernelGGL((k_step<10, 20, true, false, true, true>), grid, block, 0, s, ST_STEP_ARGS(p));
            else if (f32) hipLaunchKernelGGL((k_step<10, 20, true, false, false, true>), grid, block, 0, s, ST_STEP_ARGS(p));
            else if (sc0) hipLaunchKernelGGL((k_step<10, 20, false, false, true, true>), grid, block, 0, s, ST_STEP_ARGS(p));
            else hipLaunchKernelGGL((k_step<10, 20, false, false, false, true>), grid, block, 0, s, ST_STEP_ARGS(p));
        } else {
            if (f32) hipLaunchKernelGGL((k_step<0, 0, true, false, false, true>), grid, block, 0, s, ST_STEP_ARGS(p));
            else hipLaunchKernelGGL((k_step<0, 0, false, false, false, true>), grid, block, 0, s, ST_STEP_ARGS(p));
        }
    } else if (p.stamps && p.W == 10 && p.H == 20) {
        if (f32) hipLaunchKernelGGL((k_step<10, 20, true, true>), grid, block, 0, s, ST_STEP_ARGS(p));
        else if (sc0) hipLaunchKernelGGL((k_step<10, 20, false, true, true>), grid, block, 0, s, ST_STEP_ARGS(p));
        else hipLaunchKernelGGL((k_step<10, 20, false, true>), grid, block, 0, s, ST_STEP_ARGS(p));
    } else if (p.W == 10 && p.H == 20) {
        if (f32 && sc0) hipLaunchKernelGGL((k_step<10, 20, true, false, true>), grid, block, 0, s, ST_STEP_ARGS(p));
        else if (f32) hipLaunchKernelGGL((k_step<10, 20, true>), grid, block, 0, s, ST_STEP_ARGS(p));
        else if (sc0) hipLaunchKernelGGL((k_step<10, 20, false, false, true>), grid, block, 0, s, ST_STEP_ARGS(p));
        else hipLaunchKernelGGL((k_step<10, 20, false>), grid, block, 0, s, ST_STEP_ARGS(p));
    } else {
        if (f32) hipLaunchKernelGGL((k_step<0, 0, true>), grid, block, 0, s, ST_STEP_ARGS(p));
        else hipLaunchKernelGGL((k_step<0, 0, false>), grid, block, 0, s, ST_STEP_ARGS(p));
    }
    return hipGetLastError();
}

hipError_t launch_mt_sync(const KParams &p, hipStream_t s) {
    hipLaunchKernelGGL(k_mt_sync, dim3((unsigned)(p.stride / kWave)), dim3(kWave), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_render(const KParams &p, hipStream_t s) {
    hipLaunchKernelGGL(k_render, dim3((unsigned)(p.stride / kWave)), dim3(kWave), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_rollout(const KParams &p, hipStream_t s) {
    const bool f32 = p.obs_f32 != nullptr;
    const bool sc0 = !(p.flags & kScoringFlags);
    const int64_t wgs = p.stride / kWave;
    const dim3 grid((unsigned)wgs);
    if (wgs > 4 * (int64_t)(p.cus > 0 ? p.cus : 256) && !p.stamps) {
        const dim3 block(2 * kWave);  // logic + draw wave
        if (p.W == 10 && p.H == 20) {
            if (f32 && sc0) hipLaunchKernelGGL((k_rollout2<10, 20, true, true>), grid, block, 0, s, p);
            else if (f32) hipLaunchKernelGGL((k_rollout2<10, 20, true>), grid, block, 0, s, p);
            else if (sc0) hipLaunchKernelGGL((k_rollout2<10, 20, false, true>), grid, block, 0, s, p);
            else hipLaunchKernelGGL((k_rollout2<10, 20, false>), grid, block, 0, s, p);
        } else {
            if (f32) hipLaunchKernelGGL((k_rollout2<0, 0, true>), grid, block, 0, s, p);
            else hipLaunchKernelGGL((k_rollout2<0, 0, false>), grid, block, 0, s, p);
        }
        return hipGetLastError();
    }
    const dim3 block(3 * kWave);  // logic + draw + output wave
    if (p.stamps && p.W == 10 && p.H == 20 && !f32) {  // diagnostic phase stamps (ST_STAMPS)
        if (sc0) hipLaunchKernelGGL((k_rollout<10, 20, false, true, true>), grid, block, 0, s, p);
        else hipLaunchKernelGGL((k_rollout<10, 20, false, false, true>), grid, block, 0, s, p);
    } else if (p.W == 10 && p.H == 20) {
        if (f32 && sc0) hipLaunchKernelGGL((k_rollout<10, 20, true, true>), grid, block, 0, s, p);
        else if (f32) hipLaunchKernelGGL((k_rollout<10, 20, true>), grid, block, 0, s, p);
        else if (sc0) hipLaunchKernelGGL((k_rollout<10, 20, false, true>), grid, block, 0, s, p);
        else hipLaunchKernelGGL((k_rollout<10, 20, false>), grid, block, 0, s, p);
    } else {
        if (f32) hipLaunchKernelGGL((k_rollout<0, 0, true>), grid, block, 0, s, p);
        else hipLaunchKernelGGL((k_rollout<0, 0, false>), grid, block, 0, s, p);
    }
    return hipGetLastError();
}

// st_unwire / st_unwire_shards: the wire format (st_step_wire, above) of
// `shards` gathered blocks [shards][words][n_cap] back to packed obs
// [W][n_global], reward [n_global] and done [n_global] in global env order;
// shard r holds envs [off_r, off_r + cnt_r) at its columns 0 .. cnt_r - 1,
// the contiguous blocks of distributed.shard_range (the first n_global %
// shards shards one env more).  One env per thread, words [j][n_cap]
// coalesced across the wave, outputs coalesced.
__global__ __launch_bounds__(256) void k_unwire(int W, int H, int64_t n_global, int shards, int64_t n_cap,
                                                const uint32_t *__restrict__ wire, uint32_t *__restrict__ obs,
                                                int32_t *__restrict__ reward, uint8_t *__restrict__ done) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n_global) return;
    const int64_t base = n_global / shards, rem = n_global - base * shards;
    int64_t r, i;
    if (g < rem * (base + 1)) {
        r = g / (base + 1);
        i = g - r * (base + 1);
    } else {
        r = rem + (g - rem * (base + 1)) / base;
        i = g - rem * (base + 1) - (r - rem) * base;
    }
    const int words = (W * H + 33 + 31) / 32;
    const uint32_t hm = (1u << H) - 1u;
    const uint32_t *src = wire + r * (int64_t)words * n_cap + i;
    uint64_t acc = 0;
    int nb = 0;
    auto take = [&](int k) -> uint32_t {  // k <= 32
        if (nb < k) {
            acc |= (uint64_t)*src << nb;
            src += n_cap;
            nb += 32;
        }
        const uint32_t v = (uint32_t)acc & (k == 32 ? ~0u : (1u << k) - 1u);
        acc >>= k;
        nb -= k;
        return v;
    };
    for (int x = 0; x < W; ++x) obs[(int64_t)x * n_global + g] = take(H) & hm;
    reward[g] = (int32_t)take(32);
    done[g] = (uint8_t)take(1);
}

hipError_t launch_unwire(int W, int H, int64_t n_global, int shards, int64_t n_cap, const uint32_t *wire,
                         uint32_t *obs, int32_t *reward, uint8_t *done, hipStream_t s) {
    if (n_global <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_unwire, dim3((unsigned)((n_global + 255) / 256)), dim3(256), 0, s, W, H, n_global, shards,
                       n_cap, wire, obs, reward, done);
    return hipGetLastError();
}

hipError_t launch_obs_f32(const KParams &p, const uint32_t *obs, float *out, hipStream_t s) {
    if (p.n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_obs_f32, dim3((unsigned)((p.n + kWave - 1) / kWave)), dim3(256), 0, s, obs, out, p.n,
                       p.W, p.H);
    return hipGetLastError();
}

hipError_t launch_grayscale(const KParams &p, const uint32_t *obs, int size, int channels,
                            int as_u8, void *out, hipStream_t s) {
    if (p.n <= 0) return hipSuccess;
    // float32 rgb in sweep order (84 rgb f32 at 65,536 envs: 1,035 us against
    // 1,105 us per 2-env block; grayscale and u8 measured faster per block:
    // 356 vs 405 us, 2,072 vs 3,265 us), when a wave iteration's U 1-KB runs
    // span at most two envs and the output is 16-B aligned; else per block
    const int V = as_u8 ? 16 : 4;
    const int64_t per = (int64_t)size * size * channels;
    if (!as_u8 && channels == 3 && kWave * V * kImgRuns <= per &&
        (reinterpret_cast<uintptr_t>(out) & 15u) == 0 && (p.n * per) % V == 0) {
        const int64_t runs = (p.n * per + kWave * V - 1) / (kWave * V);
        const int64_t want = (runs + 4 * kImgRuns - 1) / (4 * kImgRuns);  // 4 waves per block
        const dim3 grid((unsigned)(want < kImgSweepGrid ? want : kImgSweepGrid)), block(256);
        if (as_u8 && channels == 3)
            hipLaunchKernelGGL((k_grayscale_sweep<uint8_t, 3>), grid, block, 0, s, obs, (uint8_t *)out, p.n, p.W,
                               p.H, size);
        else if (as_u8)
            hipLaunchKernelGGL((k_grayscale_sweep<uint8_t, 1>), grid, block, 0, s, obs, (uint8_t *)out, p.n, p.W,
                               p.H, size);
        else if (channels == 3)
            hipLaunchKernelGGL((k_grayscale_sweep<float, 3>), grid, block, 0, s, obs, (float *)out, p.n, p.W,
                               p.H, size);
        else
            hipLaunchKernelGGL((k_grayscale_sweep<float, 1>), grid, block, 0, s, obs, (float *)out, p.n, p.W,
                               p.H, size);
        return hipGetLastError();
    }
    const dim3 grid((unsigned)((p.n + kImgEnvs - 1) / kImgEnvs)), block(256);
    if (as_u8 && channels == 3)
        hipLaunchKernelGGL((k_grayscale<uint8_t, 3>), grid, block, 0, s, obs, (uint8_t *)out, p.n, p.W, p.H, size);
    else if (as_u8)
        hipLaunchKernelGGL((k_grayscale<uint8_t, 1>), grid, block, 0, s, obs, (uint8_t *)out, p.n, p.W, p.H, size);
    else if (channels == 3)
        hipLaunchKernelGGL((k_grayscale<float, 3>), grid, block, 0, s, obs, (float *)out, p.n, p.W, p.H, size);
    else
        hipLaunchKernelGGL((k_grayscale<float, 1>), grid, block, 0, s, obs, (float *)out, p.n, p.W, p.H, size);
    return hipGetLastError();
}

hipError_t launch_policy_greedy(const KParams &p, uint64_t seed, int64_t t, uint32_t explore,
                                uint8_t *out, hipStream_t s) {
    hipLaunchKernelGGL(k_policy_greedy, dim3((unsigned)(p.stride / kWave)), dim3(kWave), 0, s, p, seed, t,
                       explore, out);
    return hipGetLastError();
}

hipError_t launch_check_actions(const uint8_t *a, int64_t n, uint32_t *flag, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_check_actions, dim3((unsigned)((n + 16 * 256 - 1) / (16 * 256))), dim3(256), 0, s, a,
                       n, flag);
    return hipGetLastError();
}

hipError_t launch_gate_actions(const uint8_t *a, int64_t n, uint32_t *words, uint32_t *host, uint32_t epoch,
                               hipStream_t s) {
    // at most 64 blocks of 256 threads, 16 actions per thread and pass
    const int64_t want = (n + 16 * 256 - 1) / (16 * 256);
    const unsigned blocks = (unsigned)(want < 1 ? 1 : (want > 64 ? 64 : want));
    hipLaunchKernelGGL(k_gate_actions, dim3(blocks), dim3(256), 0, s, a, n, words, host, epoch);
    return hipGetLastError();
}

hipError_t launch_gen_actions(uint8_t *out, int64_t n, int64_t t, uint64_t seed, int64_t off,
                              hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_gen_actions, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, out, n,
                       t, seed, off);
    return hipGetLastError();
}

hipError_t launch_export(const KParams &p, int64_t env, const uint32_t *obs, const int32_t *rew,
                         const uint8_t *done, uint32_t parts, uint32_t *out, hipStream_t s) {
    hipLaunchKernelGGL(k_export, dim3(1), dim3(256), 0, s, p, env, obs, rew, done, parts, out);
    return hipGetLastError();
}

}  // namespace st
