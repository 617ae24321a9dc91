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

// One descriptor per (piece, rot): four 8-bit column records
//   bits 0-2 dx+3, bits 3-5 (top dy)+3, bits 6-7 run length-1.
// Tetromino columns are vertically contiguous runs (checked below); pieces
// with fewer than 4 columns repeat their last column (OR/AND/min idempotent).
// rot r = r applications of rotated(cclk=False) (tetris_env.py:22-26).
struct PieceTab {
    uint32_t d[28];
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
            uint32_t desc = 0, last = 0;
            int ncol = 0;
            for (int dx = -3; dx <= 3; ++dx) {
                int ymin = 99, ymax = -99, cnt = 0;
                for (int c = 0; c < 4; ++c)
                    if (cx[c] == dx) {
                        ++cnt;
                        ymin = cy[c] < ymin ? cy[c] : ymin;
                        ymax = cy[c] > ymax ? cy[c] : ymax;
                    }
                if (!cnt) continue;
                if (cnt != ymax - ymin + 1 || ymin < -3 || ymax > 3) t.ok = false;
                last = (uint32_t)(dx + 3) | ((uint32_t)(ymin + 3) << 3) | ((uint32_t)(ymax - ymin) << 6);
                desc |= last << (8 * ncol);
                ++ncol;
            }
            for (int j = ncol; j < 4; ++j) desc |= last << (8 * j);
            t.d[p * 4 + r] = desc;
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
__constant__ uint32_t c_tab[28] = {
    kTab.d[0],  kTab.d[1],  kTab.d[2],  kTab.d[3],  kTab.d[4],  kTab.d[5],  kTab.d[6],
    kTab.d[7],  kTab.d[8],  kTab.d[9],  kTab.d[10], kTab.d[11], kTab.d[12], kTab.d[13],
    kTab.d[14], kTab.d[15], kTab.d[16], kTab.d[17], kTab.d[18], kTab.d[19], kTab.d[20],
    kTab.d[21], kTab.d[22], kTab.d[23], kTab.d[24], kTab.d[25], kTab.d[26], kTab.d[27]};

// Piece table entry `lane` (lanes 0..27) materialised from immediates: no
// memory round trip at kernel entry.
__device__ __forceinline__ uint32_t tab_entry(int lane) {
    uint32_t v = 0;
#pragma unroll
    for (int j = 0; j < 28; ++j) v = lane == j ? kTab.d[j] : v;
    return v;
}

__device__ __forceinline__ int col_dx(uint32_t c) { return (int)(c & 7u) - 3; }
__device__ __forceinline__ int col_top(uint32_t c) { return (int)((c >> 3) & 7u) - 3; }
__device__ __forceinline__ int col_bot(uint32_t c) { return col_top(c) + (int)(c >> 6); }

// Bits of one piece column's cells at anchor row y; cells with y < 0 vanish
// (is_occupied skips them, tetris_env.py:32-33; _set_piece clips them, :326).
__device__ __forceinline__ uint32_t run_bits(uint32_t c, int y) {
    const int top = y + col_top(c);
    const uint32_t m = (2u << (c >> 6)) - 1u;
    return top >= 0 ? (m << top) : (m >> (-top));
}

__device__ __forceinline__ uint32_t &lcol(uint32_t *L, int x, int lane) {
    return L[(x + kPad) * kWave + lane];
}

// The four column words a descriptor touches at anchor column x (issued as
// one batch of LDS reads), and the collision / drop tests on them:
//  collides_v = is_occupied (tetris_env.py:29-36) with the floor bits and the
//    all-ones wall columns standing in for the bounds checks; cells with y < 0
//    vanish in run_bits (R2);
//  drop_v = the number of free soft_drops below a legal position, i.e.
//    hard_drop's loop count (tetris_env.py:54-59): only each column's lowest
//    cell can meet an obstacle first, and the first obstacle row is the lowest
//    set bit of (column | floor) at or below it.  A column outside the board
//    (legal only while its cells are above row 0) reads a wall and stops the
//    piece as its lowest cell would enter row 0.
__device__ __forceinline__ void read_cols(const uint32_t *L, int lane, uint32_t d, int x,
                                          uint32_t (&v)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t c = (d >> (8 * j)) & 0xFFu;
        v[j] = L[(x + col_dx(c) + kPad) * kWave + lane];
    }
}
__device__ __forceinline__ bool collides_v(uint32_t d, int y, const uint32_t (&v)[4]) {
    uint32_t hit = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) hit |= run_bits((d >> (8 * j)) & 0xFFu, y) & v[j];
    return hit != 0;
}
__device__ __forceinline__ int drop_v(uint32_t d, int y, const uint32_t (&v)[4]) {
    int dist = 1 << 20;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int yb = y + col_bot((d >> (8 * j)) & 0xFFu);
        const int s = yb + 1 > 0 ? yb + 1 : 0;
        const int k = __builtin_ctz(v[j] & (~0u << s)) - yb - 1;
        dist = k < dist ? k : dist;
    }
    return dist;
}

// _set_piece(True) (tetris_env.py:323-327): cells inside the board only.
__device__ __forceinline__ void paint(uint32_t *L, int lane, uint32_t d, int x, int y, uint32_t hmask) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t c = (d >> (8 * j)) & 0xFFu;
        atomicOr(&lcol(L, x + col_dx(c), lane), run_bits(c, y) & hmask);  // ds_or_b32
    }
}

// _set_piece(False): erase the cells (only matters on a death step, R8).
__device__ __forceinline__ void erase(uint32_t *L, int lane, uint32_t d, int x, int y, uint32_t hmask) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t c = (d >> (8 * j)) & 0xFFu;
        atomicAnd(&lcol(L, x + col_dx(c), lane), ~(run_bits(c, y) & hmask));  // ds_and_b32
    }
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

// _count_holes (tetris_env.py:218-220) for one column: empty cells below the
// topmost filled cell.
__device__ __forceinline__ int col_holes(uint32_t v, int H) {
    return v ? H - __builtin_ctz(v) - __builtin_popcount(v) : 0;
}

// ---------------------------------------------------------------- MT19937
// CPython Modules/_randommodule.c genrand_uint32 / init_by_array.
__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}
__device__ __forceinline__ uint32_t mt_mix(uint32_t a, uint32_t b) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

// Wave-cooperative twist of ONE env's 624-word state `g` (must be called by
// all 64 lanes, wave-uniformly).  The serial recurrence splits into four
// chunks whose elements only read OLD words or words of earlier chunks:
// [0,227) old | [227,454) uses [0,227) | [454,623) uses [227,396) | 623.
__device__ void coop_twist(uint32_t *g, uint32_t *S, int lane) {
    {
        uint32_t t[10];  // 624 = 9 * 64 + 48: issue all ten loads before any wait
#pragma unroll
        for (int q = 0; q < 10; ++q) {
            const int i = lane + kWave * q;
            t[q] = i < kMtN ? g[i] : 0u;
        }
#pragma unroll
        for (int q = 0; q < 10; ++q) {
            const int i = lane + kWave * q;
            if (i < kMtN) S[i] = t[q];
        }
    }
    __syncthreads();
    uint32_t v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int k = lane + kWave * q;
        if (k < 227) v[q] = S[k + 397] ^ mt_mix(S[k], S[k + 1]);
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int k = lane + kWave * q;
        if (k < 227) S[k] = v[q];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int k = 227 + lane + kWave * q;
        if (k < 454) v[q] = S[k - 227] ^ mt_mix(S[k], S[k + 1]);
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int k = 227 + lane + kWave * q;
        if (k < 454) S[k] = v[q];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        const int k = 454 + lane + kWave * q;
        if (k < 623) v[q] = S[k - 227] ^ mt_mix(S[k], S[k + 1]);
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        const int k = 454 + lane + kWave * q;
        if (k < 623) S[k] = v[q];
    }
    __syncthreads();
    if (lane == 0) S[623] = S[396] ^ mt_mix(S[623], S[0]);
    __syncthreads();
    for (int i = lane; i < kMtN; i += kWave) g[i] = S[i];
}

// _choose_shape (tetris_env.py:183-191) + the count update of _new_piece
// (:199) for every lane with `need`.  randint(1, sum(m)) = 1 + _randbelow(n)
// with rejection sampling on getrandbits(k) (Lib/random.py:239-249).
// Wave-uniform: every lane of the wave must call it.  Each round reads up to 8
// consecutive words per lane (one or two 64-B lines of the env's MT block);
// lanes whose state is exhausted are twisted cooperatively first.
// Issue the loads of the next 8 MT words of this lane's stream (used by the
// step kernel as soon as it knows the lane locks, so the round trip overlaps
// the lock-path work).
__device__ __forceinline__ void prefetch_words(const uint32_t *g, int32_t mtidx, bool want,
                                               uint32_t (&w)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
        w[j] = (want && mtidx + j < kMtN) ? __builtin_nontemporal_load(g + mtidx + j) : 0u;
}

__device__ __forceinline__ int draw_shape(bool need, int32_t (&cnt)[7], int32_t &mtidx,
                                          uint32_t *mt_wave, uint32_t *S, int lane, bool twist,
                                          const uint32_t (&pre)[8], bool have_pre) {
    int32_t maxc = cnt[0], sumc = cnt[0];
#pragma unroll
    for (int i = 1; i < 7; ++i) {
        maxc = cnt[i] > maxc ? cnt[i] : maxc;
        sumc += cnt[i];
    }
    const uint32_t n = (uint32_t)(35 + 7 * maxc - sumc);
    const int k = 32 - __builtin_clz(n);
    uint32_t *g = mt_wave + (size_t)lane * kMtN;
    bool pending = need;
    bool fresh = false;  // state twisted (and stored) by this wave in this launch
    uint32_t r = 0;
    while (__ballot(pending)) {
        if (!twist && pending && mtidx >= kMtN) mtidx = 0;  // ablation: skip the twist
        uint64_t tw = __ballot(pending && mtidx >= kMtN);
        uint32_t w[8];
        bool have = false;
        if (have_pre && pending && mtidx < kMtN) {  // words prefetched by the caller
#pragma unroll
            for (int j = 0; j < 8; ++j) w[j] = pre[j];
            have = true;
        }
        have_pre = false;
        if (tw) {
            do {
                const int l = __builtin_ctzll(tw);
                tw &= tw - 1;
                coop_twist(mt_wave + (size_t)l * kMtN, S, lane);
                if (lane == l) {  // the twisted lane takes its first words from LDS
#pragma unroll
                    for (int j = 0; j < 8; ++j) w[j] = S[j];
                    have = true;
                }
                __syncthreads();  // S is reused by the next lane's twist
            } while (tw);
            if (have) {
                mtidx = 0;
                fresh = true;
            }
        }
        if (pending && !have) {
            // A state twisted in this launch is re-read from global memory only
            // if one draw needs more than 8 of its words (p ~ 1e-3): drain our
            // stores to L2 first; the nt loads bypass the (stale) L1.
            if (__ballot(pending && fresh)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
            for (int j = 0; j < 8; ++j)
                w[j] = (mtidx + j < kMtN) ? __builtin_nontemporal_load(g + mtidx + j) : 0u;
        }
        if (pending) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (pending && mtidx < kMtN) {
                    const uint32_t y = mt_temper(w[j]) >> (32 - k);
                    ++mtidx;
                    if (y < n) {
                        pending = false;
                        r = y;
                    }
                }
            }
        }
    }
    if (!need) return 0;
    int32_t rr = (int32_t)r + 1;
    int pick = 6;
    bool found = false;
#pragma unroll
    for (int i = 0; i < 7; ++i) {
        rr -= 5 + maxc - cnt[i];
        if (!found && rr <= 0) {
            pick = i;
            found = true;
        }
    }
#pragma unroll
    for (int i = 0; i < 7; ++i) cnt[i] += (i == pick);
    return pick;
}

__device__ __forceinline__ uint32_t pack_piece(int id, int rot, int ax, int ay, int lock) {
    return (uint32_t)id | ((uint32_t)rot << 3) | ((uint32_t)ax << 5) | ((uint32_t)ay << 11) |
           ((uint32_t)lock << 17);
}

// ---------------------------------------------------------------- step
// In-kernel phase stamps (diagnostic instantiation only; MI355X guide §7).
#define ST_STAMP(i)                                                    \
    do {                                                               \
        if constexpr (STAMP) {                                         \
            __builtin_amdgcn_sched_barrier(0);                         \
            tstamp[i] = __builtin_amdgcn_s_memtime();                  \
            __builtin_amdgcn_sched_barrier(0);                         \
        }                                                              \
    } while (0)

template <int WT, int HT, bool F32, bool STAMP = false>
__global__ __launch_bounds__(kWave) void k_step(KParams p) {
    [[maybe_unused]] uint64_t tstamp[8] = {};
    ST_STAMP(0);
    // LDS: board columns L[x + kPad][lane] (walls at both ends), the staged
    // counter rows SS[r][lane] (r < 14: stats rows, 14: piece word), the MT
    // twist scratch and the piece table.
    __shared__ __attribute__((aligned(16))) uint32_t L[(kMaxW + 2 * kPad) * kWave];
    __shared__ __attribute__((aligned(16))) uint32_t SS[kHotQ * 4 * kWave];
    __shared__ uint32_t S[kMtN];
    __shared__ uint32_t T[28];
    const int W = WT ? WT : p.W;
    const int H = HT ? HT : p.H;
    const int lane = threadIdx.x;
    const int64_t e0 = (int64_t)blockIdx.x * kWave;
    const int64_t e = e0 + lane;
    const int64_t sd = p.stride;
    const bool real = e < p.n;
    const uint32_t hmask = (1u << H) - 1u;
    const uint32_t floorb = ~hmask;

    // ---- loads: 16 B per lane (a wave's slice of one SoA row is 256 B) ----
    // Unconditional (clamped) so the compiler issues them all back to back:
    // board slots past the last column land in the right-wall columns, which
    // are written after them; counter slots past row 14 land in padding row 15.
    constexpr int NBQ = ((WT ? WT : kMaxW) * 16 + kWave - 1) / kWave;  // board x4 slots
    uint4 bv[NBQ];
#pragma unroll
    for (int q = 0; q < NBQ; ++q) {
        const int i = q * kWave + lane, c = i & 15;
        const int x = (i >> 4) < W ? (i >> 4) : W - 1;
        bv[q] = *reinterpret_cast<const uint4 *>(p.board + x * sd + e0 + 4 * c);
    }
    uint4 sv[kHotQ];
#pragma unroll
    for (int q = 0; q < kHotQ; ++q) {
        const int i = q * kWave + lane, c = i & 15;
        const int r = (i >> 4) < kHotRows ? (i >> 4) : kHotRows - 1;
        const uint32_t *row = r < kStatRows ? reinterpret_cast<const uint32_t *>(p.stats) + r * sd
                                            : p.piece;
        sv[q] = *reinterpret_cast<const uint4 *>(row + e0 + 4 * c);
    }
    const uint32_t act = real ? (uint32_t)p.actions[e] : 6u;
    if (lane < 28) T[lane] = tab_entry(lane);
#pragma unroll
    for (int q = 0; q < NBQ; ++q) {
        const int i = q * kWave + lane, x = i >> 4, c = i & 15;
        uint4 v = bv[q];
        v.x |= floorb;
        v.y |= floorb;
        v.z |= floorb;
        v.w |= floorb;
        *reinterpret_cast<uint4 *>(&L[(x + kPad) * kWave + 4 * c]) = v;
    }
#pragma unroll
    for (int x = 0; x < kPad; ++x) {  // walls (after the board slots, see above)
        L[x * kWave + lane] = ~0u;
        L[(W + kPad + x) * kWave + lane] = ~0u;
    }
#pragma unroll
    for (int q = 0; q < kHotQ; ++q) {
        const int i = q * kWave + lane, c = i & 15;
        *reinterpret_cast<uint4 *>(&SS[(i >> 4) * kWave + 4 * c]) = sv[q];
    }
    __syncthreads();
    auto ss = [&](int r) -> uint32_t & { return SS[r * kWave + lane]; };

    const uint32_t pw = ss(kPieceRow);
    int32_t time = (int32_t)ss(ST_STAT_TIME);
    const int id = (int)(pw & 7u);
    int rot = (int)((pw >> 3) & 3u);
    int ax = (int)((pw >> 5) & 63u);
    int ay = (int)((pw >> 11) & 63u);
    int lock = (int)(pw >> 17);
    if constexpr (STAMP) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    ST_STAMP(1);

    // ---- action (tetris_env.py:245; value_action_map :152-160) + drop ----
    // Current and candidate descriptors and their columns are read in one
    // LDS round trip each; the collision and drop tests are then pure VALU.
    const bool tries = act == 0u || act == 1u || act == 4u || act == 5u;
    const int cx = ax + (act == 0u ? -1 : (act == 1u ? 1 : 0));
    const int cr = act == 4u ? ((rot + 1) & 3) : (act == 5u ? ((rot + 3) & 3) : rot);
    uint32_t desc = T[id * 4 + rot];
    const uint32_t cdesc = T[id * 4 + cr];
    uint32_t cur[4], cand[4];
    read_cols(L, lane, desc, ax, cur);
    read_cols(L, lane, cdesc, cx, cand);
    int d;
    if (tries && !collides_v(cdesc, ay, cand)) {
        ax = cx;
        rot = cr;
        desc = cdesc;
        d = drop_v(cdesc, ay, cand);
    } else {
        d = drop_v(desc, ay, cur);
    }
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
        if (p.flags & ST_STEP_RESET) lock = 0;
    }
    time += 1;
    int32_t rew = (p.flags & ST_REWARD_STEP) ? 1 : 0;
    bool locknow = false;
    if (d == 0) {
        lock = lock + 1 < p.lock_mod ? lock + 1 : (p.lock_mod == 1 ? 0 : (lock + 1) % p.lock_mod);
        locknow = lock == 0 && !(p.ablate & 1u);
    }
    ST_STAMP(2);
    // MT words for the piece this lock will draw: issue now, consume after the
    // lock path (every locking lane draws: a spawn, or the same-step reset's).
    int32_t mtidx = (int32_t)ss(ST_STAT_MT_INDEX);
    uint32_t pre[8];
    const bool want_pre = locknow && mtidx < kMtN && !(p.ablate & 2u);
    prefetch_words(p.mt + e * kMtN, mtidx, want_pre, pre);

    // ---- lock path (tetris_env.py:263-299) ----
    bool died = false, spawn = false;
    int32_t score = 0, lines = 0, holes = 0, height = 0, deaths = 0;
    if (locknow) {
        score = (int32_t)ss(ST_STAT_SCORE);
        lines = (int32_t)ss(ST_STAT_LINES);
        holes = (int32_t)ss(ST_STAT_HOLES);
        height = (int32_t)ss(ST_STAT_PIECE_HEIGHT);
        deaths = (int32_t)ss(ST_STAT_DEATHS);
        paint(L, lane, desc, ax, ay, hmask);
        uint32_t andv = hmask, orv = 0;
        int32_t nh = 0;
#pragma unroll 8
        for (int x = 0; x < W; ++x) {
            const uint32_t v = lcol(L, x, lane) & hmask;
            andv &= v;
            orv |= v;
            nh += col_holes(v, H);
        }
        int32_t ncl = 0;
        if (andv) {  // full rows: compact, recount
            ncl = __builtin_popcount(andv);
            orv = 0;
            nh = 0;
#pragma unroll 8
            for (int x = 0; x < W; ++x) {
                const uint32_t v = compact(lcol(L, x, lane) & hmask, andv);
                lcol(L, x, lane) = v | floorb;
                orv |= v;
                nh += col_holes(v, H);
            }
            lines += ncl;
        }
        if (p.flags & ST_ADVANCED_CLEARS) {  // :266-269, 2.5 * [0,40,100,300,1200]
            const int32_t sc = ncl == 1 ? 40 : ncl == 2 ? 100 : ncl == 3 ? 300 : ncl == 4 ? 1200 : 0;
            rew += (sc * 5) / 2;
            score += sc;
        } else if (p.flags & ST_HIGH_SCORING) {  // :270-272
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
            const int32_t old_holes = holes;
            holes = nh;
            const int32_t hgt = __builtin_popcount(orv);  // sum(np.any(board, axis=0))
            if (p.flags & ST_PENALISE_HEIGHT) {
                rew -= hgt;
            } else if (p.flags & ST_PENALISE_HEIGHT_INCREASE) {
                if (hgt > height) rew -= 10 * (hgt - height);
                height = hgt;
            }
            if (p.flags & ST_PENALISE_HOLES) rew -= 5 * holes;
            else if (p.flags & ST_PENALISE_HOLES_INCREASE) rew -= 5 * (holes - old_holes);
            spawn = true;
        }
    }
    ST_STAMP(3);

    // ---- spawn (:299 _new_piece) or same-step reset (:306-315) ----
    const bool reset_now = died && p.autoreset == ST_AUTORESET_SAME_STEP;
    const bool draw = spawn || reset_now;
    int32_t cnt[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) cnt[i] = draw ? (int32_t)ss(ST_STAT_COUNT0 + i) : 0;
    const int pick = (p.ablate & 2u) ? 0
                                      : draw_shape(draw, cnt, mtidx, p.mt + e0 * kMtN, S, lane,
                                                   !(p.ablate & 4u), pre, want_pre);
    ST_STAMP(4);
    uint32_t odesc = desc;
    int oax = ax, oay = ay;
    uint32_t pw_out = pack_piece(id, rot, ax, ay, lock);
    if (draw) pw_out = pack_piece(pick, 0, W / 2, 0, lock);
    if (spawn) {
        odesc = T[pick * 4];
        oax = W / 2;
        oay = 0;
    }

    // ---- counters back to the staged rows (tetris_env.py:253, :264-299) ----
    if (reset_now) {
        int32_t *st = p.stats + e;
        st[ST_STAT_EP_TIME * sd] = time;
        st[ST_STAT_EP_SCORE * sd] = score;
        st[ST_STAT_EP_LINES * sd] = lines;
        st[ST_STAT_EP_HOLES * sd] = holes;
        time = score = lines = holes = height = 0;
    }
    ss(ST_STAT_TIME) = (uint32_t)time;
    ss(kPieceRow) = pw_out;
    if (locknow) {
        ss(ST_STAT_SCORE) = (uint32_t)score;
        ss(ST_STAT_LINES) = (uint32_t)lines;
        ss(ST_STAT_HOLES) = (uint32_t)holes;
        ss(ST_STAT_PIECE_HEIGHT) = (uint32_t)height;
        ss(ST_STAT_DEATHS) = (uint32_t)deaths;
        ss(ST_STAT_MT_INDEX) = (uint32_t)mtidx;
        if (draw) ss(ST_STAT_COUNT0 + pick) += 1u;  // shape_counts[name] += 1, :199
    }

    // ---- observation (tetris_env.py:301-302): board + current piece ----
    paint(L, lane, odesc, oax, oay, hmask);
    __syncthreads();
    const bool wide_obs = (p.n & 3) == 0 && e0 + kWave <= p.n &&
                          (reinterpret_cast<uintptr_t>(p.obs) & 15u) == 0;
    if (p.obs && !(p.ablate & 8u)) {
        if (wide_obs) {
#pragma unroll
            for (int q = 0; q < NBQ; ++q) {
                const int i = q * kWave + lane, x = i >> 4, c = i & 15;
                if (x < W) {
                    uint4 v = *reinterpret_cast<const uint4 *>(&L[(x + kPad) * kWave + 4 * c]);
                    v.x &= hmask;
                    v.y &= hmask;
                    v.z &= hmask;
                    v.w &= hmask;
                    *reinterpret_cast<uint4 *>(p.obs + x * p.n + e0 + 4 * c) = v;
                }
            }
        } else if (real) {
            for (int x = 0; x < W; ++x) p.obs[x * p.n + e] = lcol(L, x, lane) & hmask;
        }
    }
    if (real) {
        if (p.reward) p.reward[e] = rew;
        if (p.done) p.done[e] = died ? 1 : 0;
    }
    if (F32) {
        // float32 obs [n][W][H] of the wave's envs is one contiguous block:
        // 16-B chunks, lane-consecutive, bits read back from L.
        const int64_t nreal64 = p.n - e0 < kWave ? p.n - e0 : kWave;
        const int nreal = (int)nreal64;
        const int per_env = W * H;
        const int total = nreal * per_env;
        float *out = p.obs_f32 + e0 * per_env;
        auto word = [&](int ee, int x) { return L[(x + kPad) * kWave + ee] & hmask; };
        if ((per_env & 3) == 0) {
            float4 *out4 = reinterpret_cast<float4 *>(out);
            for (int c = lane; c < total / 4; c += kWave) {
                const int f = c * 4;
                const int ee = f / per_env;
                const int rem = f - ee * per_env;
                const int x = rem / H;
                const int y = rem - x * H;
                float4 v;
                if (y + 4 <= H) {
                    const uint32_t w = word(ee, x) >> y;
                    v.x = (float)(w & 1u);
                    v.y = (float)((w >> 1) & 1u);
                    v.z = (float)((w >> 2) & 1u);
                    v.w = (float)((w >> 3) & 1u);
                } else {
                    float t4[4];
                    int xx = x, yy = y;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        t4[q] = (float)((word(ee, xx) >> yy) & 1u);
                        if (++yy == H) {
                            yy = 0;
                            ++xx;
                        }
                    }
                    v = make_float4(t4[0], t4[1], t4[2], t4[3]);
                }
                out4[c] = v;
            }
        } else {
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

    // ---- state: board = obs minus the overlay (no-op where the overlay was
    // already part of the board... see below), counters, piece ----
    // Erasing the overlaid piece yields the post-step board for every lane:
    // non-locking lanes and spawns (overlay cells were empty), and a death
    // without auto-reset (R8: _set_piece(False), tetris_env.py:303).
    __syncthreads();
    erase(L, lane, odesc, oax, oay, hmask);
    if (reset_now)
        for (int x = 0; x < W; ++x) lcol(L, x, lane) = floorb;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NBQ; ++q) {
        const int i = q * kWave + lane, x = i >> 4, c = i & 15;
        if (x < W) {
            uint4 v = *reinterpret_cast<const uint4 *>(&L[(x + kPad) * kWave + 4 * c]);
            v.x &= hmask;
            v.y &= hmask;
            v.z &= hmask;
            v.w &= hmask;
            *reinterpret_cast<uint4 *>(p.board + x * sd + e0 + 4 * c) = v;
        }
    }
#pragma unroll
    for (int q = 0; q < kHotQ; ++q) {
        const int i = q * kWave + lane, r = i >> 4, c = i & 15;
        if (r < kHotRows) {
            uint32_t *row = r < kStatRows ? reinterpret_cast<uint32_t *>(p.stats) + r * sd : p.piece;
            *reinterpret_cast<uint4 *>(row + e0 + 4 * c) =
                *reinterpret_cast<const uint4 *>(&SS[r * kWave + 4 * c]);
        }
    }
    if constexpr (STAMP) {
        ST_STAMP(6);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        ST_STAMP(7);
        if (lane == 0) {
#pragma unroll
            for (int i = 0; i < 8; ++i) p.stamps[blockIdx.x * 8 + i] = tstamp[i];
        }
    }
}

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
    int32_t mtidx = st[ST_STAT_MT_INDEX * sd];
    const uint32_t pw = p.piece[e];
    const uint32_t nopre[8] = {};
    const int pick = draw_shape(m, cnt, mtidx, p.mt + e0 * kMtN, S, lane, true, nopre, false);
    if (m) {
        st[ST_STAT_TIME * sd] = 0;
        st[ST_STAT_SCORE * sd] = 0;
        st[ST_STAT_HOLES * sd] = 0;
        st[ST_STAT_LINES * sd] = 0;
        st[ST_STAT_PIECE_HEIGHT * sd] = 0;
        st[ST_STAT_MT_INDEX * sd] = mtidx;
#pragma unroll
        for (int i = 0; i < 7; ++i) st[(ST_STAT_COUNT0 + i) * sd] = cnt[i];
        for (int x = 0; x < p.W; ++x) p.board[x * sd + e] = 0u;
        p.piece[e] = pack_piece(pick, 0, p.W / 2, 0, (int)(pw >> 17));
    }
}

// ---------------------------------------------------------------- seed
// random.seed(s): init_by_array(key = 32-bit limbs of s) (+ the first twist,
// done here so the step kernels start at index 0), and the counter values of
// TetrisEngine.__init__ (:165-181).  One lane per env, serial (one-time).
__global__ void k_seed(KParams p) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= p.stride) return;
    const uint64_t s = p.seeds[e];
    const uint32_t key[2] = {(uint32_t)s, (uint32_t)(s >> 32)};
    const int len = (s >> 32) ? 2 : 1;
    uint32_t *g = p.mt + e * kMtN;
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
    // first twist (genrand_uint32 with index == N)
    int kk = 0;
    for (; kk < kMtN - 397; ++kk) g[kk] = g[kk + 397] ^ mt_mix(g[kk], g[kk + 1]);
    for (; kk < kMtN - 1; ++kk) g[kk] = g[kk + (397 - kMtN)] ^ mt_mix(g[kk], g[kk + 1]);
    g[kMtN - 1] = g[396] ^ mt_mix(g[kMtN - 1], g[0]);

    const int64_t sd = p.stride;
    int32_t *st = p.stats + e;
    for (int r = 0; r < ST_NSTAT; ++r) st[r * sd] = 0;
    st[ST_STAT_TIME * sd] = -1;   // :165
    st[ST_STAT_SCORE * sd] = -1;  // :166
    st[ST_STAT_MT_INDEX * sd] = 0;
    for (int x = 0; x < p.W; ++x) p.board[x * sd + e] = 0u;
    p.piece[e] = pack_piece(0, 0, p.W / 2, 0, 0);
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
    const uint32_t d = c_tab[(pw & 7u) * 4 + ((pw >> 3) & 3u)];
    paint(L, lane, d, (int)((pw >> 5) & 63u), (int)((pw >> 11) & 63u), hmask);
    if (e < p.n)
        for (int x = 0; x < W; ++x) p.obs[x * p.n + e] = lcol(L, x, lane) & hmask;
}

// ---------------------------------------------------------------- misc
// packed obs [W][n] -> float32 [n][W][H] (TetrisEnv.step float32 cast, :400).
__global__ void k_obs_f32(const uint32_t *__restrict__ obs, float *__restrict__ out, int64_t n,
                          int W, int H) {
    const int64_t total = n * W * H;
    for (int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; f < total;
         f += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = f / (W * H);
        const int rem = (int)(f - e * W * H);
        const int x = rem / H;
        const int y = rem - x * H;
        out[f] = (float)((obs[x * n + e] >> y) & 1u);
    }
}

// convert_grayscale (tetris_env.py:76-114) in closed form.  The reference
// transposes the (W, H) board to (H, W), scales each cell to blk x blk, puts
// `gap` background lines before every block row/column and after the last,
// then centres the result with border (0) padding.  Pixel (r, c): r runs over
// board rows y, c over board columns x.  One thread per output pixel.
template <typename T>
__global__ void k_grayscale(const uint32_t *__restrict__ obs, T *__restrict__ out, int64_t n,
                            int W, int H, int size, int channels) {
    const int lim = W > H ? W : H;
    const int gap = size / 100 + 1;
    const int blk = (size - 2 * gap) / lim - gap;
    const int pitch = blk + gap;
    const int pr = (size - (gap + pitch * H)) / 2;  // padding_width  (axis 0 = y)
    const int pc = (size - (gap + pitch * W)) / 2;  // padding_height (axis 1 = x)
    const int64_t per = (int64_t)size * size;
    const int64_t total = n * per;
    for (int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; f < total;
         f += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = f / per;
        const int pix = (int)(f - e * per);
        const int r = pix / size - pr;
        const int c = pix - (pix / size) * size - pc;
        uint32_t v = 0;  // border_shade
        if (r >= 0 && c >= 0 && r < gap + pitch * H && c < gap + pitch * W) {
            v = 128;  // background_shade
            const int ry = r % pitch, cx = c % pitch;
            if (ry >= gap && cx >= gap) {
                const int y = r / pitch, x = c / pitch;
                if ((obs[(int64_t)x * n + e] >> y) & 1u) v = 190;  // piece_shade
            }
        }
        T *o = out + f * channels;
        for (int ch = 0; ch < channels; ++ch) o[ch] = (T)v;
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

hipError_t launch_step(const KParams &p, hipStream_t s) {
    const dim3 grid((unsigned)(p.stride / kWave)), block(kWave);
    const bool f32 = p.obs_f32 != nullptr;
    if (p.stamps && p.W == 10 && p.H == 20) {
        if (f32) hipLaunchKernelGGL((k_step<10, 20, true, true>), grid, block, 0, s, p);
        else hipLaunchKernelGGL((k_step<10, 20, false, true>), grid, block, 0, s, p);
    } else if (p.W == 10 && p.H == 20) {
        if (f32) hipLaunchKernelGGL((k_step<10, 20, true>), grid, block, 0, s, p);
        else hipLaunchKernelGGL((k_step<10, 20, false>), grid, block, 0, s, p);
    } else {
        if (f32) hipLaunchKernelGGL((k_step<0, 0, true>), grid, block, 0, s, p);
        else hipLaunchKernelGGL((k_step<0, 0, false>), grid, block, 0, s, p);
    }
    return hipGetLastError();
}

hipError_t launch_render(const KParams &p, hipStream_t s) {
    hipLaunchKernelGGL(k_render, dim3((unsigned)(p.stride / kWave)), dim3(kWave), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_obs_f32(const KParams &p, const uint32_t *obs, float *out, hipStream_t s) {
    const int64_t total = p.n * p.W * p.H;
    int64_t blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_obs_f32, dim3((unsigned)blocks), dim3(256), 0, s, obs, out, p.n, p.W, p.H);
    return hipGetLastError();
}

hipError_t launch_grayscale(const KParams &p, const uint32_t *obs, int size, int channels,
                            int as_u8, void *out, hipStream_t s) {
    const int64_t total = p.n * (int64_t)size * size;
    int64_t blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (as_u8)
        hipLaunchKernelGGL(k_grayscale<uint8_t>, dim3((unsigned)blocks), dim3(256), 0, s, obs,
                           (uint8_t *)out, p.n, p.W, p.H, size, channels);
    else
        hipLaunchKernelGGL(k_grayscale<float>, dim3((unsigned)blocks), dim3(256), 0, s, obs,
                           (float *)out, p.n, p.W, p.H, size, channels);
    return hipGetLastError();
}

hipError_t launch_gen_actions(uint8_t *out, int64_t n, int64_t t, uint64_t seed, int64_t off,
                              hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_gen_actions, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, out, n,
                       t, seed, off);
    return hipGetLastError();
}

}  // namespace st
