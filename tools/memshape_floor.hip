// Round 5 diagnostic (the empty-kernel floor is tools/launch_floor.hip's,
// 1.55 us per dependent launch): the launch-to-launch period of st_step's
// grid doing only memory work.  Back-to-back launches on one stream, HIP
// events around 4,000 of them, for (1) an empty kernel of st_step's grid, (2)
// one dependent u32 load -> store per lane, and (3) st_step's memory shape
// alone: each
// 64-env wave loads 12 board rows + 15 counter rows of its envs (SoA, 256 B
// per row and wave, the same as st_step's prologue) and stores them back
// (board + 6 counter rows, non-temporal), two waves per workgroup of 64 envs.
// Build: hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-kernarg-preload-count=6
//        tools/memshape_floor.hip -o tools/memshape_floor
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int kWave = 64;

__global__ __launch_bounds__(128) void k_empty(uint32_t *a, uint32_t *b, int64_t n) {
    if (a == nullptr && b == nullptr && n < 0) a[0] = 0;  // never true: keeps the arguments live
}

__global__ __launch_bounds__(128) void k_one(uint32_t *a, uint32_t *b, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 128 + threadIdx.x;
    if (i < n) b[i] = a[i] + 1u;
}

// one workgroup = 64 envs; wave 0 the board rows, wave 1 the counter rows
__global__ __launch_bounds__(128) void k_shape(uint32_t *board, uint32_t *stats, int64_t stride) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t e = (int64_t)blockIdx.x * kWave + lane;
    if (w == 0) {
        uint32_t v[12];
#pragma unroll
        for (int r = 0; r < 12; ++r) v[r] = board[r * stride + e];
#pragma unroll
        for (int r = 0; r < 12; ++r) __builtin_nontemporal_store(v[r] ^ 1u, &board[r * stride + e]);
    } else {
        uint32_t v[15];
#pragma unroll
        for (int r = 0; r < 15; ++r) v[r] = stats[r * stride + e];
        uint32_t x = 0;
#pragma unroll
        for (int r = 0; r < 15; ++r) x += v[r];
#pragma unroll
        for (int r = 0; r < 6; ++r) __builtin_nontemporal_store(v[r] + x, &stats[r * stride + e]);
    }
}

int main(int argc, char **argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 65536;
    const int K = 4000, WU = 200;
    hipStream_t s;
    CK(hipStreamCreate(&s));
    uint32_t *a, *b, *board, *stats;
    CK(hipMalloc(&a, n * 2 * 4));
    CK(hipMalloc(&b, n * 2 * 4));
    CK(hipMalloc(&board, n * 12 * 4));
    CK(hipMalloc(&stats, n * 19 * 4));
    CK(hipMemset(a, 0, n * 2 * 4));
    CK(hipMemset(board, 0, n * 12 * 4));
    CK(hipMemset(stats, 0, n * 19 * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const dim3 g((unsigned)(n / kWave)), blk(128);
    auto launch = [&](int kind) {
        if (kind == 0) hipLaunchKernelGGL(k_empty, g, blk, 0, s, a, b, n);
        else if (kind == 1) hipLaunchKernelGGL(k_one, dim3((unsigned)(2 * n / 128)), blk, 0, s, a, b, 2 * n);
        else hipLaunchKernelGGL(k_shape, g, blk, 0, s, board, stats, n);
    };
    for (int kind = 0; kind < 3; ++kind) {
        const char *name = kind == 0 ? "empty (grid of st_step)" : kind == 1 ? "one u32 load->store per lane"
                                                                            : "st_step memory shape";
        for (int rep = 0; rep < 3; ++rep) {
            for (int t = 0; t < WU + K; ++t) {
                if (t == WU) CK(hipEventRecord(e0, s));
                launch(kind);
            }
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            CK(hipGetLastError());
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("%s n=%lld eager rep %d: %.3f us per launch\n", name, (long long)n, rep, ms * 1e3 / K);
            fflush(stdout);
        }
        // the same K launches replayed from a hipGraph (no per-launch host
        // call: the GPU-side period)
        hipGraph_t gr;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        for (int t = 0; t < K; ++t) launch(kind);
        CK(hipStreamEndCapture(s, &gr));
        CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipEventRecord(e0, s));
            CK(hipGraphLaunch(ge, s));
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("%s n=%lld graph rep %d: %.3f us per launch\n", name, (long long)n, rep, ms * 1e3 / K);
            fflush(stdout);
        }
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(gr));
    }
    CK(hipStreamSynchronize(s));
    return 0;
}
