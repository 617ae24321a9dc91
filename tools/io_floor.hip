// io_floor.hip -- the floor under st_step at 65,536 envs: a kernel of the same
// grid (1,024 workgroups x 2 waves, 64 envs per workgroup) that moves
// st_step's compulsory bytes with its access shapes and NO game logic,
// graph-replayed back to back like bench.py:
//   empty    : launch floor of the grid
//   io1      : one round trip: read board 10 rows + counter rows 15 + action
//              + the 16-B draw-window cache (SoA, 16 B per lane), then write
//              obs 10 rows + reward + done + time + piece (non-temporal, as
//              st_step) -- every store depends on the loads
//   io2      : io1 plus st_step's second, dependent round trip: 21% of lanes
//              (st_step's lock rate) read 32 B at a data-dependent offset of
//              their env's 5,056-B MT state (331 MB array) before the stores
// Build: hipcc --offload-arch=gfx950 -O3 tools/io_floor.hip -o tools/io_floor
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int kPitch = 1264;  // MT words per env (st_internal.h kMtPitch)

__global__ __launch_bounds__(128) void k_empty(int *p) { if (p && threadIdx.x == 9999) p[0] = 1; }

__device__ __forceinline__ void st_nt(uint32_t *p, uint32_t v) { __builtin_nontemporal_store(v, p); }

template <bool TWO>
__global__ __launch_bounds__(128) void k_io(const uint32_t *__restrict__ state, const uint8_t *__restrict__ act,
                                            const uint32_t *__restrict__ mtc, const uint32_t *__restrict__ mt,
                                            uint32_t *__restrict__ out, int64_t sd) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;  // two waves per 64 envs, as st_step
    const int64_t e = (int64_t)blockIdx.x * 64 + lane;
    uint32_t acc = act[e];
    // wave 0: board rows 0..9 + counter rows 10..17; wave 1: counter rows 18..24 + cache
    const int r0 = wave ? 18 : 0, r1 = wave ? 25 : 18;
    uint32_t v[18];
#pragma unroll
    for (int i = 0; i < 18; ++i) v[i] = (r0 + i < r1) ? state[(int64_t)(r0 + i) * sd + e] : 0u;
    uint4 c = make_uint4(0, 0, 0, 0);
    if (wave) c = reinterpret_cast<const uint4 *>(mtc)[e];
#pragma unroll
    for (int i = 0; i < 18; ++i) acc ^= v[i];
    acc ^= c.x ^ c.y ^ c.z ^ c.w;
    if (TWO && wave) {
        // 21% of lanes: a dependent 32-B read inside the env's MT state
        const uint32_t h = (acc * 2654435761u) ^ (uint32_t)e * 40503u;
        if ((h & 1023u) < 217u) {
            const uint32_t off = (h >> 10) % (kPitch - 8);
            const uint4 *w = reinterpret_cast<const uint4 *>(mt + e * kPitch + (off & ~3u));
            const uint4 a = w[0], b = w[1];
            acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w;
        }
    }
    // outputs: wave 0 obs rows 0..9, wave 1 reward, done (as a word), time, piece
    const int o0 = wave ? 10 : 0, o1 = wave ? 14 : 10;
    for (int r = o0; r < o1; ++r) st_nt(out + (int64_t)r * sd + e, acc + r);
}

template <typename F>
static float time_graph(F launch, hipStream_t s, int K) {
    if (hipDeviceSynchronize() != hipSuccess) return -1.f;
    hipGraph_t g;
    hipGraphExec_t ge;
    hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
    for (int i = 0; i < K; ++i) launch();
    hipStreamEndCapture(s, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    hipGraphLaunch(ge, s);
    hipStreamSynchronize(s);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a, s);
    hipGraphLaunch(ge, s);
    hipEventRecord(b, s);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    hipGraphExecDestroy(ge);
    hipGraphDestroy(g);
    return ms * 1000.f / K;
}

int main() {
    const int64_t n = 65536, sd = n;
    uint32_t *state, *mtc, *mt, *out;
    uint8_t *act;
    CHECK(hipMalloc(&state, 25 * sd * 4));
    CHECK(hipMalloc(&mtc, sd * 16));
    CHECK(hipMalloc(&mt, (size_t)sd * kPitch * 4));
    CHECK(hipMalloc(&out, 14 * sd * 4));
    CHECK(hipMalloc(&act, sd));
    CHECK(hipMemset(state, 1, 25 * sd * 4));
    CHECK(hipMemset(mtc, 2, sd * 16));
    CHECK(hipMemset(mt, 3, (size_t)sd * kPitch * 4));
    CHECK(hipMemset(act, 1, sd));
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    const int K = 2000;
    const dim3 grid(n / 64), block(128);
    for (int rep = 0; rep < 2; ++rep) {
        float t0 = time_graph([&] { hipLaunchKernelGGL(k_empty, grid, block, 0, s, nullptr); }, s, K);
        float t1 = time_graph([&] { hipLaunchKernelGGL(k_io<false>, grid, block, 0, s, state, act, mtc, mt, out, sd); }, s, K);
        float t2 = time_graph([&] { hipLaunchKernelGGL(k_io<true>, grid, block, 0, s, state, act, mtc, mt, out, sd); }, s, K);
        printf("{\"empty_us\": %.3f, \"io1_us\": %.3f, \"io2_us\": %.3f, \"io_bytes_per_env\": "
               "{\"read\": %d, \"write\": %d, \"mt_window_locking_lanes\": 32}}\n",
               t0, t1, t2, 25 * 4 + 1 + 16, 14 * 4);
    }
    return 0;
}
