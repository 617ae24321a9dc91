// write_bw.hip -- achievable HBM write bandwidth on this part: the ceiling for
// the write-bound image / float32-obs kernels (k_grayscale writes 1.85 GB per
// 65,536-env launch with lane-consecutive 16-B non-temporal stores).
// Streams of 16-B stores, plain and non-temporal, over 1.85 GB, with 16 B per
// lane per iteration and a grid of 256 .. 8192 workgroups.
// Build: hipcc --offload-arch=gfx950 -O3 tools/write_bw.hip -o tools/write_bw
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

typedef unsigned int u4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(256) void k_write(u4 *dst, size_t n16, uint32_t seed) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
        const u4 v = {seed, (uint32_t)i, seed ^ 1u, (uint32_t)(i >> 32)};
        if (NT) __builtin_nontemporal_store(v, dst + i);
        else dst[i] = v;
    }
}

// grid-stride with U lane-consecutive chunks per thread per iteration
// (window per grid iteration = gridDim * 256 * U * 16 B)
template <int U>
__global__ __launch_bounds__(256) void k_write_u(u4 *dst, size_t n16, uint32_t seed) {
    const size_t stride = (size_t)gridDim.x * blockDim.x * U;
    for (size_t i0 = (size_t)blockIdx.x * blockDim.x * U + threadIdx.x; i0 < n16; i0 += stride) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = i0 + (size_t)u * blockDim.x;
            const u4 v = {seed, (uint32_t)i, seed ^ 1u, (uint32_t)(i >> 32)};
            if (i < n16) __builtin_nontemporal_store(v, dst + i);
        }
    }
}

// each block writes its own contiguous region of `per` 16-B chunks (the
// image kernels' block -> region mapping), lane-consecutive
template <bool NT>
__global__ __launch_bounds__(256) void k_write_blocked(u4 *dst, size_t n16, size_t per, uint32_t seed) {
    const size_t b0 = (size_t)blockIdx.x * per, b1 = b0 + per < n16 ? b0 + per : n16;
    for (size_t i = b0 + threadIdx.x; i < b1; i += blockDim.x) {
        const u4 v = {seed, (uint32_t)i, seed ^ 1u, (uint32_t)(i >> 32)};
        if (NT) __builtin_nontemporal_store(v, dst + i);
        else dst[i] = v;
    }
}

int main() {
    const size_t bytes = (size_t)65536 * 84 * 84 * 4;  // one grayscale f32 batch
    const size_t n16 = bytes / 16;
    u4 *d;
    CHECK(hipMalloc(&d, bytes));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const int R = 20;
    for (int rep = 0; rep < 2; ++rep)
        for (int nt = 0; nt < 2; ++nt)
            for (int wg : {256, 1024, 2048, 4096, 8192}) {
                for (int i = 0; i < 3; ++i) {
                    if (nt) hipLaunchKernelGGL(k_write<true>, dim3(wg), dim3(256), 0, 0, d, n16, (uint32_t)i);
                    else hipLaunchKernelGGL(k_write<false>, dim3(wg), dim3(256), 0, 0, d, n16, (uint32_t)i);
                }
                CHECK(hipEventRecord(a, 0));
                for (int i = 0; i < R; ++i) {
                    if (nt) hipLaunchKernelGGL(k_write<true>, dim3(wg), dim3(256), 0, 0, d, n16, (uint32_t)i);
                    else hipLaunchKernelGGL(k_write<false>, dim3(wg), dim3(256), 0, 0, d, n16, (uint32_t)i);
                }
                CHECK(hipEventRecord(b, 0));
                CHECK(hipEventSynchronize(b));
                float ms;
                CHECK(hipEventElapsedTime(&ms, a, b));
                const double us = ms * 1000.0 / R;
                printf("{\"nt\": %d, \"workgroups\": %d, \"bytes\": %zu, \"us\": %.1f, \"TBps\": %.3f}\n", nt, wg,
                       bytes, us, bytes / us / 1e6);
            }
    auto run_u = [&](int u, unsigned wg) -> double {
        auto go = [&](uint32_t i) {
            if (u == 1) hipLaunchKernelGGL(k_write_u<1>, dim3(wg), dim3(256), 0, 0, d, n16, i);
            else if (u == 4) hipLaunchKernelGGL(k_write_u<4>, dim3(wg), dim3(256), 0, 0, d, n16, i);
            else hipLaunchKernelGGL(k_write_u<16>, dim3(wg), dim3(256), 0, 0, d, n16, i);
        };
        for (int i = 0; i < 3; ++i) go(i);
        hipEventRecord(a, 0);
        for (int i = 0; i < R; ++i) go(i);
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        return ms * 1000.0 / R;
    };
    for (int rep = 0; rep < 2; ++rep)
        for (int u : {1, 4, 16})
            for (unsigned wg : {64u, 128u, 256u, 512u, 1024u}) {
                const double us = run_u(u, wg);
                printf("{\"sweep_u\": %d, \"workgroups\": %u, \"window_kb\": %u, \"us\": %.1f, \"TBps\": %.3f}\n",
                       u, wg, wg * 256 * u * 16 / 1024, us, bytes / us / 1e6);
            }
    // block-contiguous regions: 16 envs (the current image kernel), 4, 1, 1/4 env
    for (int rep = 0; rep < 2; ++rep)
        for (size_t env_bytes_x4 : {(size_t)64, (size_t)16, (size_t)4, (size_t)1}) {
            const size_t per = env_bytes_x4 * (84 * 84 * 4) / 4 / 16;  // 16-B chunks per block
            const unsigned grid = (unsigned)((n16 + per - 1) / per);
            for (int i = 0; i < 3; ++i)
                hipLaunchKernelGGL(k_write_blocked<true>, dim3(grid), dim3(256), 0, 0, d, n16, per, (uint32_t)i);
            CHECK(hipEventRecord(a, 0));
            for (int i = 0; i < R; ++i)
                hipLaunchKernelGGL(k_write_blocked<true>, dim3(grid), dim3(256), 0, 0, d, n16, per, (uint32_t)i);
            CHECK(hipEventRecord(b, 0));
            CHECK(hipEventSynchronize(b));
            float ms;
            CHECK(hipEventElapsedTime(&ms, a, b));
            const double us = ms * 1000.0 / R;
            printf("{\"blocked_envs\": %.2f, \"workgroups\": %u, \"us\": %.1f, \"TBps\": %.3f}\n",
                   env_bytes_x4 / 4.0, grid, us, bytes / us / 1e6);
        }
    CHECK(hipFree(d));
    return 0;
}
