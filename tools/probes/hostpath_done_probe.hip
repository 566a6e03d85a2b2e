// Host path of large calls, fourth probe: how the host learns that a registered
// call's last kernel (the copy into the caller's result block, csrc/rle_dropin.cpp) has finished.
// Per size, medians of 40 reps in microseconds, each a copy kernel of n bytes from device memory
// into a registered host block:
//   sync       hipStreamSynchronize (the library's form)
//   flag_poll  a one-lane kernel after the copy stores a word into mapped pinned memory behind a
//              system-scope release; the host polls it (no workgroup of the copy itself releases)
//   event      hipEventRecord + hipEventSynchronize
// The block is checked after each form.
// build: hipcc -O2 --offload-arch=gfx950 tools/probes/hostpath_done_probe.hip -o build/hostpath_done_probe
#include <hip/hip_runtime.h>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                     \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
template <class F>
static double med(F f, int reps = 40) {
    for (int r = 0; r < 5; ++r) f();
    std::vector<double> t;
    for (int r = 0; r < reps; ++r) {
        const double t0 = now_us();
        f();
        t.push_back(now_us() - t0);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

__global__ __launch_bounds__(256) void kcopy(uint4* __restrict__ dst, const uint4* __restrict__ src, size_t n16) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) dst[i] = src[i];
}
__global__ void flag_kernel(uint32_t* flag, uint32_t v) {
    __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void fill_kernel(uint8_t* d, size_t n, uint8_t v) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        d[i] = (uint8_t)(v + i);
}

int main() {
    hipStream_t s;
    CK(hipStreamCreate(&s));
    uint32_t* hflag = nullptr;
    CK(hipHostMalloc((void**)&hflag, 64, hipHostMallocMapped));
    uint32_t* dflag = nullptr;
    CK(hipHostGetDevicePointer((void**)&dflag, hflag, 0));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    printf("%9s %7s %9s %7s %s\n", "bytes", "sync", "flag_poll", "event", "check");
    uint32_t seq = 0;
    for (size_t n : {262144ul, 1048576ul, 4194304ul}) {
        uint8_t* h = (uint8_t*)malloc(n + 16) + 16;
        memset(h, 0, n);
        CK(hipHostRegister(h, n, hipHostRegisterMapped));
        void* dh = nullptr;
        CK(hipHostGetDevicePointer(&dh, h, 0));
        uint8_t* d = nullptr;
        CK(hipMalloc(&d, n));
        hipLaunchKernelGGL(fill_kernel, dim3(256), dim3(256), 0, s, d, n, (uint8_t)(n >> 10));
        CK(hipStreamSynchronize(s));
        const int grid = (int)std::min<size_t>(1024, (n / 16 + 255) / 256);
        int bad = 0;
        auto check = [&] {
            for (size_t i = 0; i < n; i += 4093)
                if (h[i] != (uint8_t)((n >> 10) + i)) { ++bad; break; }
        };
        const double t_sync = med([&] {
            hipLaunchKernelGGL(kcopy, dim3(grid), dim3(256), 0, s, (uint4*)dh, (const uint4*)d, n / 16);
            CK(hipStreamSynchronize(s));
        });
        check();
        const double t_flag = med([&] {
            const uint32_t v = ++seq;
            hipLaunchKernelGGL(kcopy, dim3(grid), dim3(256), 0, s, (uint4*)dh, (const uint4*)d, n / 16);
            hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(1), 0, s, dflag, v);
            while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != v) __builtin_ia32_pause();
        });
        CK(hipStreamSynchronize(s));
        check();
        const double t_ev = med([&] {
            hipLaunchKernelGGL(kcopy, dim3(grid), dim3(256), 0, s, (uint4*)dh, (const uint4*)d, n / 16);
            CK(hipEventRecord(ev, s));
            CK(hipEventSynchronize(ev));
        });
        check();
        printf("%9zu %7.1f %9.1f %7.1f %s\n", n, t_sync, t_flag, t_ev, bad ? "MISMATCH" : "ok");
        CK(hipHostUnregister(h));
        CK(hipFree(d));
        free(h - 16);
    }
    return 0;
}
