// pmc_calib.hip -- calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for
// the access shapes the step kernel uses (MI355X_MICROARCH.md §HBM: FETCH_SIZE
// is calibrated only for 16-B/lane streams; "calibrate on a known byte count
// in your own access pattern before trusting an absolute").
//
// Each kernel streams a 512 MiB buffer (2x the Infinity Cache) once:
//   rd4  : 4 B/lane coalesced loads   (the step kernel's SoA loads)
//   wr4  : 4 B/lane coalesced stores  (the step kernel's SoA stores)
//   rd16 : 16 B/lane loads            (the guide's calibrated shape)
// Build: hipcc --offload-arch=gfx950 -O3 tools/pmc_calib.hip -o tools/pmc_calib
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void rd4(const unsigned *__restrict__ in, unsigned *__restrict__ sink, size_t n) {
    unsigned acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc ^= in[i];
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void wr4(unsigned *__restrict__ out, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        out[i] = (unsigned)i;
}

__global__ void rd16(const uint4 *__restrict__ in, unsigned *__restrict__ sink, size_t n4) {
    unsigned acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = in[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
    const size_t bytes = (size_t)512 << 20, n = bytes / 4;
    unsigned *a = nullptr, *b = nullptr, *sink = nullptr;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess ||
        hipMalloc(&sink, 64) != hipSuccess) {
        fprintf(stderr, "alloc failed\n");
        return 1;
    }
    (void)hipMemset(a, 1, bytes);
    (void)hipMemset(b, 2, bytes);
    const dim3 grid(4096), block(256);
    for (int it = 0; it < 3; ++it) {
        hipLaunchKernelGGL(rd4, grid, block, 0, 0, a, sink, n);
        hipLaunchKernelGGL(wr4, grid, block, 0, 0, b, n);
        hipLaunchKernelGGL(rd16, grid, block, 0, 0, (const uint4 *)a, sink, n / 4);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("{\"bytes_per_launch\": %zu}\n", bytes);
    return 0;
}
