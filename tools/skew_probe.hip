// skew_probe.hip -- when does each XCD start a kernel's waves?  Each wave
// records s_memrealtime (100 MHz, chip-wide) at entry and exit plus its
// XCC_ID; the body spins ~4 us (about one step's wave life).  Graph-replayed
// back to back like bench.py; prints per-XCD median start offsets of the last
// replay for several grid shapes.
// Build: hipcc --offload-arch=gfx950 -O3 tools/skew_probe.hip -o tools/skew_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

template <int LDS_WORDS>
__global__ void k_probe(uint64_t *rec, int spin_ticks) {
    __shared__ uint32_t pad[LDS_WORDS > 0 ? LDS_WORDS : 1];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    if (LDS_WORDS > 0) pad[threadIdx.x % (LDS_WORDS > 0 ? LDS_WORDS : 1)] = threadIdx.x;
    uint64_t t = t0;
    while (t - t0 < (uint64_t)spin_ticks) t = __builtin_amdgcn_s_memrealtime();
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if ((threadIdx.x & 63) == 0) {
        rec[wave * 4 + 0] = t0;
        rec[wave * 4 + 1] = __builtin_amdgcn_s_memrealtime();
        rec[wave * 4 + 2] = __builtin_amdgcn_s_getreg(0xF814) & 0xF;  // XCC_ID
        rec[wave * 4 + 3] = LDS_WORDS > 0 ? pad[0] : 0;
    }
}

template <int LDS_WORDS>
static int run(const char *name, int blocks, int threads, int spin) {
    const int waves = blocks * threads / 64;
    uint64_t *rec;
    CHECK(hipMalloc(&rec, (size_t)waves * 4 * sizeof(uint64_t)));
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    hipGraph_t g;
    hipGraphExec_t ge;
    CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(k_probe<LDS_WORDS>, dim3(blocks), dim3(threads), 0, s, rec, spin);
    CHECK(hipStreamEndCapture(s, &g));
    CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CHECK(hipGraphLaunch(ge, s));
    CHECK(hipStreamSynchronize(s));
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a, s);
    CHECK(hipGraphLaunch(ge, s));
    hipEventRecord(b, s);
    CHECK(hipEventSynchronize(b));
    float ms;
    hipEventElapsedTime(&ms, a, b);
    std::vector<uint64_t> h((size_t)waves * 4);
    CHECK(hipMemcpy(h.data(), rec, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
    uint64_t t_min = ~0ull, e_max = 0;
    for (int w = 0; w < waves; ++w) {
        t_min = std::min(t_min, h[w * 4]);
        e_max = std::max(e_max, h[w * 4 + 1]);
    }
    printf("{\"config\": \"%s\", \"blocks\": %d, \"threads\": %d, \"us_per_kernel\": %.3f, \"span_ns\": %llu, \"xcd_start_median_ns\": [",
           name, blocks, threads, ms * 1000.f / 20, (unsigned long long)((e_max - t_min) * 10));
    for (int x = 0; x < 8; ++x) {
        std::vector<uint64_t> st;
        for (int w = 0; w < waves; ++w)
            if ((int)h[w * 4 + 2] == x) st.push_back(h[w * 4] - t_min);
        std::sort(st.begin(), st.end());
        printf("%s%llu", x ? ", " : "", st.empty() ? 0ull : (unsigned long long)(st[st.size() / 2] * 10));
    }
    printf("]}\n");
    hipGraphExecDestroy(ge);
    hipGraphDestroy(g);
    hipFree(rec);
    return 0;
}

int main() {
    // st_step's shape (1,024 workgroups of 2 waves, ~17.5 KB LDS each) against
    // fewer, larger workgroups carrying the same waves (round 4: does the
    // dispatch ramp scale with the workgroup count?), each wave spinning about
    // one st_step wave life (2.8 us)
    const int spin = 280;
    int rc = 0;
    for (int rep = 0; rep < 2; ++rep) {
        rc |= run<4480>("2 waves/WG, 17.5 KB LDS (st_step)", 1024, 128, spin);
        rc |= run<8960>("4 waves/WG, 35 KB LDS", 512, 256, spin);
        rc |= run<17920>("8 waves/WG, 70 KB LDS", 256, 512, spin);
        rc |= run<0>("2 waves/WG, no LDS", 1024, 128, spin);
        rc |= run<0>("4 waves/WG, no LDS", 512, 256, spin);
        rc |= run<4480>("2 waves/WG, 17.5 KB LDS, no spin", 1024, 128, 0);
        rc |= run<8960>("4 waves/WG, 35 KB LDS, no spin", 512, 256, 0);
    }
    return rc;
}
