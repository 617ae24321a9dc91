// launch_cost.hip -- host time per kernel launch through the HIP launch APIs
// (the st_step loop issues one launch per env-step; at the bench's K = 20 the
// host issue rate, ~4.4 us per ctypes st_step call, is as slow as the kernel).
// An empty kernel taking a KParams-sized struct by value, 2,000 launches per
// API, asynchronous (the queue does not fill), host wall time per call.
//
// build: hipcc -O3 --offload-arch=gfx950 -o tools/launch_cost tools/launch_cost.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <chrono>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 1;                                                                \
        }                                                                            \
    } while (0)

struct Args {  // the size of st::KParams
    uint64_t w[22];
};

__global__ void k_empty(Args a) {
    if (a.w[0] == 12345u && threadIdx.x == 1024) a.w[1] = 0;  // never true; keeps the argument live
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    Args a{};
    const dim3 grid(1024), block(128);
    const int N = 2000;
    hipFunction_t f = nullptr;
    CK(hipGetFuncBySymbol(&f, reinterpret_cast<const void *>(&k_empty)));
    size_t asz = sizeof(a);
    void *extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &asz, HIP_LAUNCH_PARAM_END};
    void *kargs[] = {&a};
    for (int rep = 0; rep < 2; ++rep) {
        double t0, t1;
        // 1. triple-chevron (hipLaunchKernelGGL)
        CK(hipStreamSynchronize(s));
        t0 = now_us();
        for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_empty, grid, block, 0, s, a);
        t1 = now_us();
        CK(hipStreamSynchronize(s));
        const double chevron = (t1 - t0) / N;
        // 2. hipLaunchKernel (argument pointer array)
        t0 = now_us();
        for (int i = 0; i < N; ++i) CK(hipLaunchKernel(reinterpret_cast<const void *>(&k_empty), grid, block, kargs, 0, s));
        t1 = now_us();
        CK(hipStreamSynchronize(s));
        const double lk = (t1 - t0) / N;
        // 3. hipModuleLaunchKernel with the packed argument buffer
        t0 = now_us();
        for (int i = 0; i < N; ++i)
            CK(hipModuleLaunchKernel(f, grid.x, 1, 1, block.x, 1, 1, 0, s, nullptr, extra));
        t1 = now_us();
        CK(hipStreamSynchronize(s));
        const double mod = (t1 - t0) / N;
        // 4. hipExtLaunchKernel
        t0 = now_us();
        for (int i = 0; i < N; ++i)
            CK(hipExtLaunchKernel(reinterpret_cast<const void *>(&k_empty), grid, block, kargs, 0, s, nullptr, nullptr, 0));
        t1 = now_us();
        CK(hipStreamSynchronize(s));
        const double ext = (t1 - t0) / N;
        // 5. device time: back-to-back empty kernels, events
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < N; ++i) CK(hipModuleLaunchKernel(f, grid.x, 1, 1, block.x, 1, 1, 0, s, nullptr, extra));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        // 6. wake-up: one empty launch, then hipStreamSynchronize, host time
        double wsum = 0;
        for (int i = 0; i < 200; ++i) {
            CK(hipStreamSynchronize(s));
            t0 = now_us();
            CK(hipModuleLaunchKernel(f, grid.x, 1, 1, block.x, 1, 1, 0, s, nullptr, extra));
            CK(hipStreamSynchronize(s));
            wsum += now_us() - t0;
        }
        printf("{\"rep\": %d, \"host_us_per_launch\": {\"hipLaunchKernelGGL\": %.3f, \"hipLaunchKernel\": %.3f, "
               "\"hipModuleLaunchKernel\": %.3f, \"hipExtLaunchKernel\": %.3f}, \"device_us_per_empty_kernel\": %.3f, "
               "\"launch_plus_sync_roundtrip_us\": %.2f, \"HIP_FORCE_DEV_KERNARG\": \"%s\"}\n",
               rep, chevron, lk, mod, ext, ms * 1e3 / N, wsum / 200, getenv("HIP_FORCE_DEV_KERNARG") ? getenv("HIP_FORCE_DEV_KERNARG") : "");
    }
    return 0;
}
