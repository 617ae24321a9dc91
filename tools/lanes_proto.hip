// lanes_proto.hip -- A/B of the two board layouts for the step's logic
// (VERDICT r2 "next" #3; BASELINE north_star: "staging each board's rows ...
// and reducing with wavefront ballot/popcount").  Timing study, not product
// code: the same simplified step (no MT19937 -- the spawned piece comes from a
// per-env LCG; everything else as TetrisEngine.step, tetris_env.py:243-304:
// action + collision (:29-36, :39-73), hard/soft drop, gravity, lock, line
// clear with compaction (:205-216), holes (:218-220) / height, death + reset)
// in two layouts, checked against each other bit for bit, then timed:
//
//   A  one env per lane (the engine's layout): the board's column words in
//      LDS [x][lane] with wall columns, collision / drop / full rows by
//      per-lane loops over the piece's 4 columns and the board's 10;
//   B  16 lanes per env (north_star): lane c holds board column c in a
//      register (c >= W idle), the piece's cells per column computed per
//      lane, collision by wave ballot, drop distance / full rows / holes /
//      height by DPP reductions over the env's 16 lanes; per-env scalars
//      replicated in its 16 lanes.  4 envs per wave, no LDS.
//
// Modes: rollout (K steps in one launch, state in registers / LDS) and
// single-step launches (state in HBM: [W][N] board, piece / LCG / counters).
//
// build: hipcc -O3 --offload-arch=gfx950 -o tools/lanes_proto tools/lanes_proto.hip
// run:   tools/lanes_proto [N=65536] [K=100] [launches=20]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

constexpr int W = 10, H = 20, PAD = 4, WAVE = 64;
constexpr uint32_t HMASK = (1u << H) - 1u, FLOORB = ~HMASK;

// tetris_env.py:10-19 (T,J,L,Z,S,I,O); descriptor per (piece, rot): m = the 4
// column records' cells (byte j: bit dy+3), g = 6 bits per record: dx+3,
// bottom dy+3; pieces with < 4 columns repeat the last record
constexpr int kShapes[7][4][2] = {
    {{0, 0}, {-1, 0}, {1, 0}, {0, -1}},  {{0, 0}, {-1, 0}, {0, -1}, {0, -2}},
    {{0, 0}, {1, 0}, {0, -1}, {0, -2}},  {{0, 0}, {-1, 0}, {0, -1}, {1, -1}},
    {{0, 0}, {-1, -1}, {0, -1}, {1, 0}}, {{0, 0}, {0, -1}, {0, -2}, {0, -3}},
    {{0, 0}, {0, -1}, {-1, 0}, {-1, -1}},
};
struct Tab {
    uint32_t m[28], g[28];
};
constexpr Tab make_tab() {
    Tab t{};
    for (int p = 0; p < 7; ++p) {
        int cx[4] = {}, cy[4] = {};
        for (int c = 0; c < 4; ++c) cx[c] = kShapes[p][c][0], cy[c] = kShapes[p][c][1];
        for (int r = 0; r < 4; ++r) {
            uint32_t m = 0, g = 0, lm = 0, lg = 0;
            int n = 0;
            for (int dx = -3; dx <= 3; ++dx) {
                int ymax = -99, cnt = 0;
                uint32_t bits = 0;
                for (int c = 0; c < 4; ++c)
                    if (cx[c] == dx) {
                        ++cnt;
                        ymax = cy[c] > ymax ? cy[c] : ymax;
                        bits |= 1u << (cy[c] + 3);
                    }
                if (!cnt) continue;
                lm = bits;
                lg = (uint32_t)(dx + 3) | ((uint32_t)(ymax + 3) << 3);
                m |= lm << (8 * n);
                g |= lg << (6 * n);
                ++n;
            }
            for (int j = n; j < 4; ++j) m |= lm << (8 * j), g |= lg << (6 * j);
            t.m[p * 4 + r] = m;
            t.g[p * 4 + r] = g;
            for (int c = 0; c < 4; ++c) {
                const int i = cx[c], j = cy[c];
                cx[c] = j;
                cy[c] = -i;
            }
        }
    }
    return t;
}
constexpr Tab kTab = make_tab();
__constant__ uint32_t c_m[28] = {kTab.m[0], kTab.m[1], kTab.m[2], kTab.m[3], kTab.m[4], kTab.m[5], kTab.m[6],
                                 kTab.m[7], kTab.m[8], kTab.m[9], kTab.m[10], kTab.m[11], kTab.m[12], kTab.m[13],
                                 kTab.m[14], kTab.m[15], kTab.m[16], kTab.m[17], kTab.m[18], kTab.m[19],
                                 kTab.m[20], kTab.m[21], kTab.m[22], kTab.m[23], kTab.m[24], kTab.m[25],
                                 kTab.m[26], kTab.m[27]};
__constant__ uint32_t c_g[28] = {kTab.g[0], kTab.g[1], kTab.g[2], kTab.g[3], kTab.g[4], kTab.g[5], kTab.g[6],
                                 kTab.g[7], kTab.g[8], kTab.g[9], kTab.g[10], kTab.g[11], kTab.g[12], kTab.g[13],
                                 kTab.g[14], kTab.g[15], kTab.g[16], kTab.g[17], kTab.g[18], kTab.g[19],
                                 kTab.g[20], kTab.g[21], kTab.g[22], kTab.g[23], kTab.g[24], kTab.g[25],
                                 kTab.g[26], kTab.g[27]};

__device__ __forceinline__ int pdx(uint32_t g, int j) { return (int)((g >> (6 * j)) & 7u) - 3; }
__device__ __forceinline__ int pbot(uint32_t g, int j) { return (int)((g >> (6 * j + 3)) & 7u) - 3; }
__device__ __forceinline__ uint32_t pbits(uint32_t m, int j, int y) { return (((m >> (8 * j)) & 0xFFu) << y) >> 3; }

__device__ __forceinline__ uint32_t hash_action(uint32_t t, uint32_t e) {
    uint64_t z = ((uint64_t)t << 32) ^ e ^ 0x5EEDull;
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return (uint32_t)((z ^ (z >> 31)) % 7ull);
}
__device__ __forceinline__ uint32_t lcg(uint32_t s) { return s * 1664525u + 1013904223u; }

// state in HBM (single-step mode) and the outputs of a run
struct State {
    uint32_t *board;  // [W][N]
    uint32_t *piece;  // [N] id | rot << 3 | ax << 5 | ay << 11
    uint32_t *rng;    // [N]
    uint32_t *cs;     // [N] checksum of every step's reward / lines / holes / height / done
    int n;
};

// one step's scalar tail shared by both layouts: reward, checksum, spawn
struct Scal {
    int id, rot, ax, ay;
    uint32_t rng, cs;
};

// ------------------------------------------------------------------ layout A
template <bool ROLL>
__global__ __launch_bounds__(WAVE) void k_lane(State s, int t0, int K) {
    __shared__ uint32_t L[(W + 2 * PAD) * WAVE];
    const int lane = threadIdx.x;
    const int e = blockIdx.x * WAVE + lane;
    const bool real = e < s.n;
    const int ec = real ? e : s.n - 1;
    auto col = [&](int x) -> uint32_t & { return L[(x + PAD) * WAVE + lane]; };
    for (int x = 0; x < W; ++x) col(x) = s.board[(size_t)x * s.n + ec] | FLOORB;
    for (int x = 0; x < PAD; ++x) L[x * WAVE + lane] = ~0u, L[(W + PAD + x) * WAVE + lane] = ~0u;
    const uint32_t pw = s.piece[ec];
    Scal q{(int)(pw & 7u), (int)((pw >> 3) & 3u), (int)((pw >> 5) & 63u), (int)((pw >> 11) & 63u), s.rng[ec],
           s.cs[ec]};
    for (int t = 0; t < K; ++t) {
        const uint32_t act = hash_action(t0 + t, e);
        const bool tries = act == 0u || act == 1u || act == 4u || act == 5u;
        const int cx = q.ax + (act == 0u ? -1 : (act == 1u ? 1 : 0));
        const int cr = act == 4u ? ((q.rot + 1) & 3) : (act == 5u ? ((q.rot + 3) & 3) : q.rot);
        uint32_t dm = c_m[q.id * 4 + q.rot], dg = c_g[q.id * 4 + q.rot];
        const uint32_t cm = c_m[q.id * 4 + cr], cg = c_g[q.id * 4 + cr];
        uint32_t cur[4], cand[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            cur[j] = col(q.ax + pdx(dg, j));
            cand[j] = col(cx + pdx(cg, j));
        }
        uint32_t hit = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) hit |= pbits(cm, j, q.ay) & cand[j];
        const bool ok = tries && hit == 0;
        if (ok) {
            q.ax = cx;
            q.rot = cr;
            dm = cm;
            dg = cg;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) cur[j] = ok ? cand[j] : cur[j];
        int d = 1 << 20;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int yb = q.ay + pbot(dg, j);
            const int sh = yb + 1 > 0 ? yb + 1 : 0;
            const int k = __builtin_ctz(cur[j] & (~0u << sh)) - yb - 1;
            d = k < d ? k : d;
        }
        if (act == 2u) {
            q.ay += d;
            d = 0;
        } else if (act == 3u && d > 0) {
            q.ay += 1;
            d -= 1;
        }
        if (d > 0) {
            q.ay += 1;
            d -= 1;
        }
        int32_t rew = 0, lines = 0, holes = 0, height = 0;
        bool died = false;
        if (d == 0) {  // lock
#pragma unroll
            for (int j = 0; j < 4; ++j) atomicOr(&col(q.ax + pdx(dg, j)), pbits(dm, j, q.ay) & HMASK);
            uint32_t andv = ~0u, orv = 0, sctz = 0, spop = 0;
#pragma unroll
            for (int x = 0; x < W; ++x) {
                const uint32_t v = col(x);
                andv &= v;
                orv |= v;
                sctz += __builtin_ctz(v);
                spop += __builtin_popcount(v);
            }
            andv &= HMASK;
            if (andv) {
                lines = __builtin_popcount(andv);
                orv = sctz = spop = 0;
                uint32_t c[W];
#pragma unroll
                for (int x = 0; x < W; ++x) c[x] = col(x) & HMASK;
                uint32_t full = andv;
                while (full) {
                    const int r = __builtin_ctz(full);
                    full &= full - 1u;
                    const uint32_t above = (1u << r) - 1u, keep = ~(above | (1u << r));
#pragma unroll
                    for (int x = 0; x < W; ++x) c[x] = (c[x] & keep) | ((c[x] & above) << 1);
                }
#pragma unroll
                for (int x = 0; x < W; ++x) {
                    const uint32_t v = c[x] | FLOORB;
                    col(x) = v;
                    orv |= v;
                    sctz += __builtin_ctz(v);
                    spop += __builtin_popcount(v);
                }
            }
            orv &= HMASK;
            holes = W * H - (int32_t)sctz - ((int32_t)spop - W * (32 - H));
            height = __builtin_popcount(orv);
            rew = 100 * lines;
            died = orv & 1u;
            if (died) {
                rew = -100;
#pragma unroll
                for (int x = 0; x < W; ++x) col(x) = FLOORB;
            }
            q.rng = lcg(q.rng);
            q.id = (int)((q.rng >> 16) % 7u);
            q.rot = 0;
            q.ax = W / 2;
            q.ay = 0;
        }
        q.cs = q.cs * 31u + (uint32_t)(rew + 7 * lines + 13 * holes + 17 * height + (died ? 1000 : 0));
    }
    if (real) {
        for (int x = 0; x < W; ++x) s.board[(size_t)x * s.n + e] = col(x) & HMASK;
        s.piece[e] = (uint32_t)q.id | ((uint32_t)q.rot << 3) | ((uint32_t)q.ax << 5) | ((uint32_t)q.ay << 11);
        s.rng[e] = q.rng;
        s.cs[e] = q.cs;
    }
}

// ------------------------------------------------------------------ layout B
// reductions over the 16 lanes of an env (DPP within a row of 16 lanes)
template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, false);
}
#define RED16(OP, x)                              \
    do {                                          \
        x = OP(x, dpp<0xB1>(x)); /* quad xor 1 */ \
        x = OP(x, dpp<0x4E>(x)); /* quad xor 2 */ \
        x = OP(x, dpp<0x141>(x)); /* half mirror */ \
        x = OP(x, dpp<0x140>(x)); /* row mirror */  \
    } while (0)
__device__ __forceinline__ uint32_t op_and(uint32_t a, uint32_t b) { return a & b; }
__device__ __forceinline__ uint32_t op_or(uint32_t a, uint32_t b) { return a | b; }
__device__ __forceinline__ uint32_t op_add(uint32_t a, uint32_t b) { return a + b; }
__device__ __forceinline__ uint32_t op_min(uint32_t a, uint32_t b) { return (int)a < (int)b ? a : b; }

template <bool ROLL>
__global__ __launch_bounds__(WAVE) void k_col(State s, int t0, int K) {
    const int lane = threadIdx.x;
    const int c = lane & 15;                   // this lane's board column
    const int e = blockIdx.x * 4 + (lane >> 4);  // 4 envs per wave
    const bool real = e < s.n;
    const int ec = real ? e : s.n - 1;
    const bool inb = c < W;
    const int shift = lane & 48;  // the env's 16-lane group in a ballot
    uint32_t colw = inb ? (s.board[(size_t)c * s.n + ec] | FLOORB) : 0u;
    const uint32_t pw = s.piece[ec];
    Scal q{(int)(pw & 7u), (int)((pw >> 3) & 3u), (int)((pw >> 5) & 63u), (int)((pw >> 11) & 63u), s.rng[ec],
           s.cs[ec]};
    // this lane's cells of descriptor (m, g) at (x0, y), the drop limit of its
    // column, and the out-of-board records (every lane computes those alike)
    auto cells = [&](uint32_t m, uint32_t g, int x0, int y) {
        uint32_t b = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) b |= (x0 + pdx(g, j) == c) ? pbits(m, j, y) : 0u;
        return b;
    };
    auto oob_hit = [&](uint32_t m, uint32_t g, int x0, int y) {
        bool h = false;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int x = x0 + pdx(g, j);
            h |= (x < 0 || x >= W) && pbits(m, j, y) != 0u;
        }
        return h;
    };
    for (int t = 0; t < K; ++t) {
        const uint32_t act = hash_action(t0 + t, e);
        const bool tries = act == 0u || act == 1u || act == 4u || act == 5u;
        const int cx = q.ax + (act == 0u ? -1 : (act == 1u ? 1 : 0));
        const int cr = act == 4u ? ((q.rot + 1) & 3) : (act == 5u ? ((q.rot + 3) & 3) : q.rot);
        uint32_t dm = c_m[q.id * 4 + q.rot], dg = c_g[q.id * 4 + q.rot];
        const uint32_t cm = c_m[q.id * 4 + cr], cg = c_g[q.id * 4 + cr];
        const bool lhit = inb && (cells(cm, cg, cx, q.ay) & colw) != 0u;
        const bool any = ((__ballot(lhit) >> shift) & 0xFFFFull) != 0ull || oob_hit(cm, cg, cx, q.ay);
        const bool ok = tries && !any;
        if (ok) {
            q.ax = cx;
            q.rot = cr;
            dm = cm;
            dg = cg;
        }
        // drop distance: this column's (the record at this column, if any),
        // min over the env's lanes and the out-of-board records
        int k = 1 << 20;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int x = q.ax + pdx(dg, j);
            const int yb = q.ay + pbot(dg, j);
            const int sh = yb + 1 > 0 ? yb + 1 : 0;
            const uint32_t v = (x < 0 || x >= W) ? ~0u : colw;
            const int kj = __builtin_ctz(v & (~0u << sh)) - yb - 1;
            const bool mine = (x < 0 || x >= W) ? (c == 0) : (x == c);  // out-of-board records: lane 0
            k = mine && kj < k ? kj : k;
        }
        uint32_t ku = (uint32_t)k;
        RED16(op_min, ku);
        int d = (int)ku;
        if (act == 2u) {
            q.ay += d;
            d = 0;
        } else if (act == 3u && d > 0) {
            q.ay += 1;
            d -= 1;
        }
        if (d > 0) {
            q.ay += 1;
            d -= 1;
        }
        int32_t rew = 0, lines = 0, holes = 0, height = 0;
        bool died = false;
        if (d == 0) {  // lock: every lane of the env together
            if (inb) colw |= cells(dm, dg, q.ax, q.ay) & HMASK;
            uint32_t andv = inb ? colw : ~0u;
            RED16(op_and, andv);
            andv &= HMASK;
            if (andv) {
                lines = __builtin_popcount(andv);
                uint32_t v = colw & HMASK, full = andv;
                while (full) {
                    const int r = __builtin_ctz(full);
                    full &= full - 1u;
                    const uint32_t above = (1u << r) - 1u, keep = ~(above | (1u << r));
                    v = (v & keep) | ((v & above) << 1);
                }
                if (inb) colw = v | FLOORB;
            }
            uint32_t orv = inb ? colw & HMASK : 0u;
            uint32_t hl = inb ? (uint32_t)(H - (int)__builtin_ctz(colw) - __builtin_popcount(colw & HMASK)) : 0u;
            RED16(op_or, orv);
            RED16(op_add, hl);
            holes = (int32_t)hl;
            height = __builtin_popcount(orv);
            rew = 100 * lines;
            died = orv & 1u;
            if (died) {
                rew = -100;
                if (inb) colw = FLOORB;
            }
            q.rng = lcg(q.rng);
            q.id = (int)((q.rng >> 16) % 7u);
            q.rot = 0;
            q.ax = W / 2;
            q.ay = 0;
        }
        q.cs = q.cs * 31u + (uint32_t)(rew + 7 * lines + 13 * holes + 17 * height + (died ? 1000 : 0));
    }
    if (real) {
        if (inb) s.board[(size_t)c * s.n + e] = colw & HMASK;
        if (c == 0) {
            s.piece[e] = (uint32_t)q.id | ((uint32_t)q.rot << 3) | ((uint32_t)q.ax << 5) | ((uint32_t)q.ay << 11);
            s.rng[e] = q.rng;
            s.cs[e] = q.cs;
        }
    }
}

// ------------------------------------------------------------------ host
struct Buf {
    State s;
    void alloc(int n) {
        s.n = n;
        CK(hipMalloc(&s.board, (size_t)W * n * 4));
        CK(hipMalloc(&s.piece, (size_t)n * 4));
        CK(hipMalloc(&s.rng, (size_t)n * 4));
        CK(hipMalloc(&s.cs, (size_t)n * 4));
    }
    void init() {
        std::vector<uint32_t> p(s.n), r(s.n);
        for (int e = 0; e < s.n; ++e) {
            r[e] = 12345u + 7919u * (uint32_t)e;
            p[e] = (uint32_t)(e % 7) | ((uint32_t)(W / 2) << 5);
        }
        CK(hipMemset(s.board, 0, (size_t)W * s.n * 4));
        CK(hipMemset(s.cs, 0, (size_t)s.n * 4));
        CK(hipMemcpy(s.piece, p.data(), (size_t)s.n * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(s.rng, r.data(), (size_t)s.n * 4, hipMemcpyHostToDevice));
    }
    std::vector<uint32_t> dump() {
        std::vector<uint32_t> o((size_t)(W + 3) * s.n);
        CK(hipMemcpy(o.data(), s.board, (size_t)W * s.n * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(o.data() + (size_t)W * s.n, s.piece, (size_t)s.n * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(o.data() + (size_t)(W + 1) * s.n, s.rng, (size_t)s.n * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(o.data() + (size_t)(W + 2) * s.n, s.cs, (size_t)s.n * 4, hipMemcpyDeviceToHost));
        return o;
    }
};

template <typename F>
static float time_it(F f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();  // warm-up
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms / reps;
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 65536;
    const int K = argc > 2 ? atoi(argv[2]) : 100;
    const int NL = argc > 3 ? atoi(argv[3]) : 20;
    Buf A, B;
    A.alloc(n);
    B.alloc(n);
    const dim3 ga((n + WAVE - 1) / WAVE), gb((n + 3) / 4);
    // correctness: the two layouts agree bit for bit after 3 rollouts of K
    // steps and 50 single steps (boards, pieces, LCGs, checksums)
    A.init();
    B.init();
    for (int r = 0; r < 3; ++r) {
        hipLaunchKernelGGL(k_lane<true>, ga, dim3(WAVE), 0, 0, A.s, r * K, K);
        hipLaunchKernelGGL(k_col<true>, gb, dim3(WAVE), 0, 0, B.s, r * K, K);
    }
    for (int t = 0; t < 50; ++t) {
        hipLaunchKernelGGL(k_lane<false>, ga, dim3(WAVE), 0, 0, A.s, 3 * K + t, 1);
        hipLaunchKernelGGL(k_col<false>, gb, dim3(WAVE), 0, 0, B.s, 3 * K + t, 1);
    }
    CK(hipDeviceSynchronize());
    const auto da = A.dump(), db = B.dump();
    size_t diff = 0;
    for (size_t i = 0; i < da.size(); ++i) diff += da[i] != db[i];
    uint64_t dead = 0;
    std::vector<uint32_t> cs(da.begin() + (size_t)(W + 2) * n, da.end());
    for (uint32_t v : cs) dead += v != 0;
    printf("{\"n\": %d, \"K\": %d, \"agree\": %s, \"words_differing\": %zu, \"envs_with_nonzero_checksum\": %llu",
           n, K, diff == 0 ? "true" : "false", diff, (unsigned long long)dead);
    // timing
    A.init();
    B.init();
    int t0 = 0;
    const float ra = time_it([&] { hipLaunchKernelGGL(k_lane<true>, ga, dim3(WAVE), 0, 0, A.s, t0, K); t0 += K; }, NL);
    t0 = 0;
    const float rb = time_it([&] { hipLaunchKernelGGL(k_col<true>, gb, dim3(WAVE), 0, 0, B.s, t0, K); t0 += K; }, NL);
    t0 = 0;
    const float sa = time_it([&] { hipLaunchKernelGGL(k_lane<false>, ga, dim3(WAVE), 0, 0, A.s, t0++, 1); }, 1000);
    t0 = 0;
    const float sb = time_it([&] { hipLaunchKernelGGL(k_col<false>, gb, dim3(WAVE), 0, 0, B.s, t0++, 1); }, 1000);
    printf(", \"rollout_us_per_step\": {\"A_lane_per_env\": %.4f, \"B_16_lanes_per_env\": %.4f}"
           ", \"single_step_us\": {\"A_lane_per_env\": %.3f, \"B_16_lanes_per_env\": %.3f}}\n",
           ra * 1e3 / K, rb * 1e3 / K, sa * 1e3, sb * 1e3);
    return diff == 0 ? 0 : 2;
}
