// floor_bench.hip -- what a step kernel of this shape costs before any game
// logic: launch floor of a 1024-wave grid and the pure HBM I/O of one step
// (the step kernel's own 16-B/lane SoA reads and writes), graph-replayed like
// bench.py.  Build: hipcc --offload-arch=gfx950 -O3 tools/floor_bench.hip -o tools/floor_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void k_empty(int *p) { if (p && threadIdx.x == 9999) p[0] = 1; }

// rows_in x4 reads, rows_out x4 writes per wave (each row = 256 B per wave)
template <int RIN, int ROUT>
__global__ __launch_bounds__(256) void k_io(const uint32_t *__restrict__ in, uint32_t *__restrict__ out, int64_t sd) {
    const int lane = threadIdx.x & 63;
    const int64_t e0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) - lane;
    constexpr int QI = (RIN * 16 + 63) / 64, QO = (ROUT * 16 + 63) / 64;
    uint4 v[QI];
#pragma unroll
    for (int q = 0; q < QI; ++q) {
        const int i = q * 64 + lane, r = (i >> 4) < RIN ? (i >> 4) : RIN - 1, c = i & 15;
        v[q] = *reinterpret_cast<const uint4 *>(in + r * sd + e0 + 4 * c);
    }
    uint4 acc = v[0];
#pragma unroll
    for (int q = 1; q < QI; ++q) { acc.x ^= v[q].x; acc.y ^= v[q].y; acc.z ^= v[q].z; acc.w ^= v[q].w; }
#pragma unroll
    for (int q = 0; q < QO; ++q) {
        const int i = q * 64 + lane, r = i >> 4, c = i & 15;
        if (r < ROUT) *reinterpret_cast<uint4 *>(out + r * sd + e0 + 4 * c) = acc;
    }
}

template <typename F>
static float time_graph(F launch, hipStream_t s, int K) {
    if (hipDeviceSynchronize() != hipSuccess) return -1.f;
    hipGraph_t g; hipGraphExec_t ge;
    hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
    for (int i = 0; i < K; ++i) launch();
    hipStreamEndCapture(s, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    hipGraphLaunch(ge, s); hipStreamSynchronize(s);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    hipEventRecord(a, s); hipGraphLaunch(ge, s); hipEventRecord(b, s); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    hipGraphExecDestroy(ge); hipGraphDestroy(g);
    return ms * 1000.f / K;
}

int main() {
    const int64_t n = 65536, sd = n;
    uint32_t *in, *out;
    // rows: k_io<RIN, ROUT> reads rows [0, RIN) of `in`, writes rows [0, ROUT) of `out`
    constexpr int kInRows = 32, kOutRows = 40;
    static_assert(25 <= kInRows && 36 <= kOutRows, "buffer rows");
    CHECK(hipMalloc(&in, kInRows * sd * 4));
    CHECK(hipMalloc(&out, kOutRows * sd * 4));
    CHECK(hipMemset(in, 1, kInRows * sd * 4));
    hipStream_t s; CHECK(hipStreamCreate(&s));
    const int K = 2000;
    for (int bs : {64, 256}) {
        const dim3 grid(n / bs), block(bs);
        float t0 = time_graph([&] { hipLaunchKernelGGL(k_empty, grid, block, 0, s, nullptr); }, s, K);
        float t1 = time_graph([&] { hipLaunchKernelGGL((k_io<1, 1>), grid, block, 0, s, in, out, sd); }, s, K);
        float t2 = time_graph([&] { hipLaunchKernelGGL((k_io<25, 36>), grid, block, 0, s, in, out, sd); }, s, K);
        float t3 = time_graph([&] { hipLaunchKernelGGL((k_io<25, 1>), grid, block, 0, s, in, out, sd); }, s, K);
        printf("{\"block\": %d, \"empty_us\": %.3f, \"io_1r1w_us\": %.3f, \"io_25r36w_us\": %.3f, \"io_25r1w_us\": %.3f, "
               "\"io_25r36w_GBs\": %.1f}\n", bs, t0, t1, t2, t3, (61.0 * 256 * n / 64) / (t2 * 1e3));
    }
    return 0;
}
