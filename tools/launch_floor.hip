// launch_floor.hip -- cost of a dependent launch of an EMPTY kernel per grid
// shape, back to back on one stream, eager and graph-replayed: does the
// 1.55 us boundary under st_step (1,024 workgroups x 128 threads) depend on
// the number or size of the workgroups?
// Build: hipcc --offload-arch=gfx950 -O3 tools/launch_floor.hip -o tools/launch_floor
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ __launch_bounds__(1024) void k_empty(int *p) { if (p && threadIdx.x == 9999) p[0] = 1; }

// the same with st_step's LDS footprint class (dynamic LDS requested)
__global__ __launch_bounds__(1024) void k_empty_lds(int *p) {
    extern __shared__ int s[];
    if (p && threadIdx.x == 9999) p[0] = s[0];
}

static float time_eager(dim3 g, dim3 b, size_t lds, hipStream_t s, int K) {
    for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(lds ? k_empty_lds : k_empty, g, b, lds, s, nullptr);
    hipStreamSynchronize(s);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, s);
    for (int i = 0; i < K; ++i) hipLaunchKernelGGL(lds ? k_empty_lds : k_empty, g, b, lds, s, nullptr);
    hipEventRecord(e1, s);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return ms * 1000.f / K;
}

static float time_graph(dim3 g, dim3 b, size_t lds, hipStream_t s, int K) {
    hipGraph_t gr;
    hipGraphExec_t ge;
    hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
    for (int i = 0; i < K; ++i) hipLaunchKernelGGL(lds ? k_empty_lds : k_empty, g, b, lds, s, nullptr);
    hipStreamEndCapture(s, &gr);
    hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0);
    hipGraphLaunch(ge, s);
    hipStreamSynchronize(s);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, s);
    hipGraphLaunch(ge, s);
    hipEventRecord(e1, s);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    hipGraphExecDestroy(ge);
    hipGraphDestroy(gr);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return ms * 1000.f / K;
}

int main(int argc, char **argv) {
    // "eager": eager launches only (a run under rocprofv3 --kernel-trace: the
    // traced duration of an empty kernel is the tracer's per-dispatch share)
    const bool eager_only = argc > 1 && argv[1][0] == 'e';
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    const int K = 2000;
    struct { int wg, th; } shapes[] = {{1, 64}, {256, 128}, {1024, 64}, {1024, 128}, {512, 256},
                                       {256, 512}, {128, 1024}, {2048, 64}, {2048, 128}, {4096, 128}};
    for (int rep = 0; rep < 2; ++rep)
        for (auto sh : shapes)
            for (size_t lds : {(size_t)0, (size_t)16384}) {
                const float e = time_eager(dim3(sh.wg), dim3(sh.th), lds, s, K);
                const float g = eager_only ? 0.f : time_graph(dim3(sh.wg), dim3(sh.th), lds, s, K);
                printf("{\"workgroups\": %d, \"threads\": %d, \"lds\": %zu, \"eager_us\": %.3f, \"graph_us\": %.3f}\n",
                       sh.wg, sh.th, lds, e, g);
            }
    CHECK(hipDeviceSynchronize());
    return 0;
}
