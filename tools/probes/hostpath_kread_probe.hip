// Host path of large calls, third probe: the inbound leg as a kernel that reads
// the caller's registered pages over PCIe, against the DMA the library uses (csrc/rle_dropin.cpp
// compress_registered: hipMemcpyAsync from the registered input, then the segmented kernels).
// Per size, medians of 40 reps in microseconds (each includes its stream sync):
//   h2d        hipMemcpyAsync registered -> device
//   h2d_k      the same, then an empty kernel on the stream (the DMA-to-kernel hand-over)
//   kread_G    a copy kernel of G workgroups x 256 lanes (16 B per lane per step) reading the
//              registered input through its device address into device memory
//   kread_G_k  the same, then the empty kernel
//   per-call reg: the same two with the input registered and unregistered around each transfer
// build: hipcc -O2 --offload-arch=gfx950 tools/probes/hostpath_kread_probe.hip -o build/hostpath_kread_probe
#include <hip/hip_runtime.h>
#include <algorithm>
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

// 16 B per lane per step, grid-strided; a 4-deep unroll keeps more loads in flight per lane
__global__ __launch_bounds__(256) void kread(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        const uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
        dst[i] = a;
        dst[i + stride] = b;
        dst[i + 2 * stride] = c;
        dst[i + 3 * stride] = d;
    }
    for (; i < n16; i += stride) dst[i] = src[i];
}
__global__ void empty_kernel() {}

int main() {
    hipStream_t s;
    CK(hipStreamCreate(&s));
    printf("%9s %7s %7s", "bytes", "h2d", "h2d_k");
    const int grids[] = {64, 256, 1024};
    for (int g : grids) printf("  kread_%-4d kread_%d_k", g, g);
    printf("\n");
    for (size_t n : {262144ul, 1048576ul, 4194304ul}) {
        uint8_t* h = (uint8_t*)malloc(n + 16) + 16;   // (malloc's alignment, as a caller's buffer)
        for (size_t i = 0; i < n; ++i) h[i] = (uint8_t)(i * 131 + 7);
        CK(hipHostRegister(h, n, hipHostRegisterMapped | hipHostRegisterReadOnly));
        void* dh = nullptr;
        CK(hipHostGetDevicePointer(&dh, h, 0));
        uint8_t* d = nullptr;
        CK(hipMalloc(&d, n));
        const double t_h2d = med([&] {
            CK(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s));
            CK(hipStreamSynchronize(s));
        });
        const double t_h2dk = med([&] {
            CK(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s));
            hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
            CK(hipStreamSynchronize(s));
        });
        printf("%9zu %7.1f %7.1f", n, t_h2d, t_h2dk);
        for (int g : grids) {
            const double t_k = med([&] {
                hipLaunchKernelGGL(kread, dim3(g), dim3(256), 0, s, (const uint4*)dh, (uint4*)d, n / 16);
                CK(hipStreamSynchronize(s));
            });
            const double t_kk = med([&] {
                hipLaunchKernelGGL(kread, dim3(g), dim3(256), 0, s, (const uint4*)dh, (uint4*)d, n / 16);
                hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
                CK(hipStreamSynchronize(s));
            });
            printf("  %10.1f %9.1f", t_k, t_kk);
        }
        // per call: register, transfer, a kernel after it, unregister (the library's registered calls)
        CK(hipHostUnregister(h));
        const double t_rdma = med([&] {
            CK(hipHostRegister(h, n, hipHostRegisterMapped | hipHostRegisterReadOnly));
            CK(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s));
            hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
            CK(hipStreamSynchronize(s));
            CK(hipHostUnregister(h));
        });
        double t_rk[3];
        for (int gi = 0; gi < 3; ++gi)
            t_rk[gi] = med([&] {
                void* dp = nullptr;
                CK(hipHostRegister(h, n, hipHostRegisterMapped | hipHostRegisterReadOnly));
                CK(hipHostGetDevicePointer(&dp, h, 0));
                hipLaunchKernelGGL(kread, dim3(grids[gi]), dim3(256), 0, s, (const uint4*)dp, (uint4*)d, n / 16);
                hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
                CK(hipStreamSynchronize(s));
                CK(hipHostUnregister(h));
            });
        printf("  | per-call reg: dma_k %.1f kread_k %.1f / %.1f / %.1f\n", t_rdma, t_rk[0], t_rk[1], t_rk[2]);
        CK(hipHostRegister(h, n, hipHostRegisterMapped | hipHostRegisterReadOnly));
        // check the last copy
        std::vector<uint8_t> back(n);
        CK(hipMemcpy(back.data(), d, n, hipMemcpyDeviceToHost));
        if (memcmp(back.data(), h, n)) printf("MISMATCH at %zu bytes\n", n);
        CK(hipHostUnregister(h));
        CK(hipFree(d));
        free(h - 16);
    }
    return 0;
}
