// Dispatch-ramp probe (gfx950): how long does the dispatcher take to start every wave of a grid
// shaped like the codec's one-round launches?  Each wave's lane 0 records s_memrealtime (100 MHz)
// first thing; the host prints the spread of start times (percentiles, us from the first start)
// for several shapes (workgroups x threads, static LDS per workgroup).
// build: hipcc --offload-arch=gfx950 -O3 tools/probes/dispatch_probe.hip -o build/dispatch_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

template <int kThreads, int kLds>
__global__ __launch_bounds__(kThreads) void probe(unsigned long long* out, unsigned spin) {
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    __shared__ uint8_t lds[kLds > 0 ? kLds : 1];
    const unsigned lane = threadIdx.x & 63, w = blockIdx.x * (kThreads / 64) + threadIdx.x / 64;
    if (kLds > 0) lds[threadIdx.x] = (uint8_t)t;
    unsigned long long e = t;
    while (e - t < spin) e = __builtin_amdgcn_s_memrealtime();
    if (kLds > 0) __syncthreads();
    if (lane == 0) out[w] = t + (kLds > 0 ? lds[(threadIdx.x + 64) % kThreads] & 0 : 0);
}

// the codec kernels' other resources: ~56 VGPRs, 336-byte kernargs, ~40 KB of code
struct BigArgs {
    unsigned long long pad[40];
};
template <int kThreads, int kLds, int kVgpr, int kCode>
__global__ __launch_bounds__(kThreads) void probe2(unsigned long long* out, unsigned spin, BigArgs ba) {
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    __shared__ uint8_t lds[kLds > 0 ? kLds : 1];
    const unsigned lane = threadIdx.x & 63, w = blockIdx.x * (kThreads / 64) + threadIdx.x / 64;
    if (kLds > 0) lds[threadIdx.x] = (uint8_t)t;
    if (kVgpr) asm volatile("" ::: "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12",
                            "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25",
                            "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38",
                            "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51",
                            "v52", "v53", "v54", "v55");
    if (kCode && spin == 12345u) {   // never taken: code size only
        asm volatile(".rept 10000\n\tv_add_u32 v1, v1, v2\n\t.endr" ::: "v1", "v2");
    }
    unsigned long long e = t;
    while (e - t < spin) e = __builtin_amdgcn_s_memrealtime();
    if (kLds > 0) __syncthreads();
    if (lane == 0) out[w] = t + (ba.pad[blockIdx.x % 40] & 0);
}

template <int kThreads, int kLds, int kVgpr = -1, int kCode = 0>
void run(const char* name, unsigned wgs, unsigned spin) {
    const unsigned waves = wgs * (kThreads / 64);
    unsigned long long* d;
    hipMalloc(&d, waves * 8);
    std::vector<unsigned long long> h(waves);
    for (int rep = 0; rep < 4; ++rep) {
        hipMemset(d, 0, waves * 8);
        hipDeviceSynchronize();
        if (kVgpr < 0) hipLaunchKernelGGL((probe<kThreads, kLds>), dim3(wgs), dim3(kThreads), 0, 0, d, spin);
        else hipLaunchKernelGGL((probe2<kThreads, kLds, (kVgpr > 0), kCode>), dim3(wgs), dim3(kThreads), 0, 0, d, spin, BigArgs{});
        hipDeviceSynchronize();
        hipMemcpy(h.data(), d, waves * 8, hipMemcpyDeviceToHost);
        std::sort(h.begin(), h.end());
        auto p = [&](double q) { return (h[(size_t)(q * (waves - 1))] - h[0]) / 100.0; };
        if (rep) printf("%-34s waves %5u  start spread us: p10 %.2f p50 %.2f p90 %.2f max %.2f\n", name, waves, p(0.1),
                        p(0.5), p(0.9), p(1.0));
    }
    hipFree(d);
}

int main() {
    run<256, 0>("1024 x 256, no LDS", 1024, 0);
    run<256, 34816>("1024 x 256, 34.8 KB LDS", 1024, 0);
    run<256, 34816>("1024 x 256, 34.8 KB LDS, 2us spin", 1024, 200);
    run<64, 8704>("4096 x 64, 8.7 KB LDS", 4096, 0);
    run<1024, 139264>("256 x 1024, 136 KB LDS", 256, 0);
    run<512, 69632>("512 x 512, 68 KB LDS", 512, 0);
    run<256, 0>("2048 x 256, no LDS (2 rounds? 8/CU)", 2048, 0);
    run<256, 34816, 0, 0>("1024 x 256, 34.8 KB, big kernarg", 1024, 0);
    run<256, 34816, 1, 0>("1024 x 256, 34.8 KB, kernarg, 56 VGPR", 1024, 0);
    run<256, 34816, 0, 1>("1024 x 256, 34.8 KB, kernarg, 40 KB code", 1024, 0);
    run<256, 34816, 1, 1>("1024 x 256, 34.8 KB, all three", 1024, 0);
    return 0;
}
