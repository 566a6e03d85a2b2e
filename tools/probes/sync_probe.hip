// Completion-latency probe (round 4, host path): how long does one tiny launch take from the host's
// point of view when the host learns of its completion (a) from hipStreamSynchronize, (b) from a flag
// the kernel writes into mapped host memory behind a system-scope release fence, (c) the same flag
// with only an s_waitcnt before it (no L2 write-back)?  The kernel reads 4 KiB of mapped input and
// writes 4 KiB of mapped output (a drop-in small call's traffic), one wave.  Each mode: 2000 calls,
// median and mean microseconds per call.
// build: hipcc --offload-arch=gfx950 -O3 tools/probes/sync_probe.hip -o build/sync_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <chrono>
#include <vector>

template <int kMode>   // 0: no flag; 1: flag behind a system release fence; 2: flag behind s_waitcnt only
__global__ void call_kernel(const uint4* __restrict__ in, uint4* __restrict__ out, volatile uint32_t* flag,
                            uint32_t token) {
    const uint32_t lane = threadIdx.x;
    for (uint32_t i = lane; i < 256; i += 64) {
        uint4 v = in[i];
        v.x ^= token;
        out[i] = v;
    }
    if (kMode == 1) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // system scope
        if (lane == 0) __hip_atomic_store(flag, token, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else if (kMode == 2) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_store(flag, token, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <int kMode>
void run(const char* name, hipStream_t s, uint4* h_in, uint4* d_in, uint4* h_out, uint4* d_out, uint32_t* h_flag,
         uint32_t* d_flag) {
    std::vector<double> t;
    uint32_t bad = 0;
    for (int it = 0; it < 2200; ++it) {
        const uint32_t token = 0x1000u + (uint32_t)it;
        for (int i = 0; i < 256; ++i) h_in[i] = make_uint4(i, it, 7, 9);
        __atomic_store_n(h_flag, 0u, __ATOMIC_RELAXED);
        const double t0 = now_us();
        hipLaunchKernelGGL(call_kernel<kMode>, dim3(1), dim3(64), 0, s, d_in, d_out, d_flag, token);
        if (kMode == 0) {
            (void)hipStreamSynchronize(s);
        } else {
            uint64_t spins = 0;
            while (__atomic_load_n((volatile uint32_t*)h_flag, __ATOMIC_ACQUIRE) != token) {
                if (++spins > 200000000ull) break;   // ~seconds: never expected
            }
        }
        const double t1 = now_us();
        for (int i = 0; i < 256; ++i)
            if (h_out[i].x != ((uint32_t)i ^ token) || h_out[i].y != (uint32_t)it) ++bad;
        if (it >= 200) t.push_back(t1 - t0);
        if (kMode != 0 && (it & 63) == 63) (void)hipStreamSynchronize(s);   // keep the queue bounded
    }
    (void)hipStreamSynchronize(s);
    std::sort(t.begin(), t.end());
    double sum = 0;
    for (double x : t) sum += x;
    printf("{\"mode\": \"%s\", \"median_us\": %.2f, \"mean_us\": %.2f, \"p10_us\": %.2f, \"p90_us\": %.2f, \"bad_words\": %u}\n",
           name, t[t.size() / 2], sum / t.size(), t[t.size() / 10], t[t.size() * 9 / 10], bad);
}

int main() {
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
    uint4 *h_in, *h_out, *d_in, *d_out;
    uint32_t *h_flag, *d_flag;
    if (hipHostMalloc((void**)&h_in, 4096, hipHostMallocMapped) != hipSuccess ||
        hipHostMalloc((void**)&h_out, 4096, hipHostMallocMapped) != hipSuccess ||
        hipHostMalloc((void**)&h_flag, 64, hipHostMallocMapped) != hipSuccess)
        return 1;
    (void)hipHostGetDevicePointer((void**)&d_in, h_in, 0);
    (void)hipHostGetDevicePointer((void**)&d_out, h_out, 0);
    (void)hipHostGetDevicePointer((void**)&d_flag, h_flag, 0);
    run<0>("hipStreamSynchronize", s, h_in, d_in, h_out, d_out, h_flag, d_flag);
    run<1>("flag after system release fence", s, h_in, d_in, h_out, d_out, h_flag, d_flag);
    run<2>("flag after s_waitcnt vmcnt(0)", s, h_in, d_in, h_out, d_out, h_flag, d_flag);
    run<0>("hipStreamSynchronize (again)", s, h_in, d_in, h_out, d_out, h_flag, d_flag);
    return 0;
}
