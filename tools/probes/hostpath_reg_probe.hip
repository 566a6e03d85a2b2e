// Host path of large calls, second probe: transfers that leave out the CPU's
// copies.  The caller's input and the result block are registered with the runtime for the call
// (hipHostRegister), the input travels by one DMA, and the device pass writes the result straight
// into the registered result block over PCIe.  Per size, medians of 40 reps in microseconds:
//   reg        hipHostRegister + hipHostGetDevicePointer of a heap buffer already touched
//   unreg      hipHostUnregister of it
//   reg_u      the same for a pointer 16 bytes past a page start (malloc's alignment)
//   h2d_reg    hipMemcpyAsync registered -> device + sync
//   k_to_reg   copy kernel device -> registered host buffer + sync
//   k_to_pin   copy kernel device -> mapped pinned buffer + sync
//   rd_pin     memcpy out of a pinned buffer the device has just written (the staged path's last copy)
//   chain      register in + out, DMA in, device pass writing into the registered out, sync,
//              unregister both (one call's transfers with no CPU copy)
//   chain_pg   pageable DMA in, device pass, pageable DMA out (the library's direct staging)
// build: hipcc -O2 --offload-arch=gfx950 tools/probes/hostpath_reg_probe.hip -o build/hostpath_reg_probe
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
template <class F>
static double med(F f, int reps = 40) {
    for (int r = 0; r < 5; ++r) f();
    std::vector<double> t;
    for (int r = 0; r < reps; ++r) {
        const double a = now_us();
        f();
        t.push_back(now_us() - a);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}
#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

__global__ void __launch_bounds__(256) copy16(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) dst[i] = src[i];
}
static void kcopy(const void* s, void* d, size_t n, hipStream_t st, int grid) {
    const size_t n16 = n / 16, need = (n16 + 255) / 256;
    const int g = (size_t)grid > need ? (int)need : grid;
    hipLaunchKernelGGL(copy16, dim3(g), dim3(256), 0, st, (const uint4*)s, (uint4*)d, n16);
}

int main() {
    const size_t kMax = 4u << 20, kPage = 4096;
    uint8_t *d_in, *d_out, *h_pin, *dh_pin;
    CK(hipMalloc(&d_in, kMax));
    CK(hipMalloc(&d_out, kMax));
    CK(hipHostMalloc(&h_pin, kMax, hipHostMallocMapped));
    CK(hipHostGetDevicePointer((void**)&dh_pin, h_pin, 0));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint8_t* in = (uint8_t*)aligned_alloc(kPage, kMax + kPage);
    uint8_t* out = (uint8_t*)aligned_alloc(kPage, kMax + kPage);
    std::vector<uint8_t> back(kMax);
    for (size_t i = 0; i < kMax + kPage; ++i) in[i] = (uint8_t)((i * 2654435761u) >> 13), out[i] = 0;
    printf("%8s %6s %6s %6s %8s %8s %8s %7s %7s %8s\n", "bytes", "reg", "unreg", "reg_u", "h2d_reg", "k_to_reg",
           "k_to_pin", "rd_pin", "chain", "chain_pg");
    for (size_t n : {262144ul, 1048576ul, 4194304ul}) {
        void* dp = nullptr;
        double tr = 0, tu = 0;
        {
            std::vector<double> a, b;
            for (int r = 0; r < 45; ++r) {
                const double t0 = now_us();
                CK(hipHostRegister(out, n, hipHostRegisterMapped));
                CK(hipHostGetDevicePointer(&dp, out, 0));
                const double t1 = now_us();
                CK(hipHostUnregister(out));
                const double t2 = now_us();
                if (r >= 5) a.push_back(t1 - t0), b.push_back(t2 - t1);
            }
            std::sort(a.begin(), a.end());
            std::sort(b.begin(), b.end());
            tr = a[a.size() / 2];
            tu = b[b.size() / 2];
        }
        const double tru = med([&] {
            CK(hipHostRegister(out + 16, n, hipHostRegisterMapped));
            CK(hipHostGetDevicePointer(&dp, out + 16, 0));
            CK(hipHostUnregister(out + 16));
        });
        CK(hipHostRegister(in, n, hipHostRegisterMapped));
        const double h2d = med([&] { CK(hipMemcpyAsync(d_in, in, n, hipMemcpyHostToDevice, s)); CK(hipStreamSynchronize(s)); });
        CK(hipHostUnregister(in));
        CK(hipHostRegister(out, n, hipHostRegisterMapped));
        CK(hipHostGetDevicePointer(&dp, out, 0));
        const double kreg = med([&] { kcopy(d_in, dp, n, s, 1024); CK(hipStreamSynchronize(s)); });
        CK(hipHostUnregister(out));
        const double kpin = med([&] { kcopy(d_in, dh_pin, n, s, 1024); CK(hipStreamSynchronize(s)); });
        const double rd = med([&] {
            kcopy(d_in, dh_pin, n, s, 1024);
            CK(hipStreamSynchronize(s));
            const double a = now_us();
            memcpy(back.data(), h_pin, n);
            return now_us() - a;
        });
        // rd above includes the kernel; time the memcpy alone
        std::vector<double> rds;
        for (int r = 0; r < 45; ++r) {
            kcopy(d_in, dh_pin, n, s, 1024);
            CK(hipStreamSynchronize(s));
            const double a = now_us();
            memcpy(back.data(), h_pin, n);
            if (r >= 5) rds.push_back(now_us() - a);
        }
        std::sort(rds.begin(), rds.end());
        (void)rd;
        const double rdm = rds[rds.size() / 2];
        memset(out, 0, n);
        const double chain = med([&] {
            void *din = nullptr, *dout = nullptr;
            CK(hipHostRegister(in + 16, n, hipHostRegisterMapped));
            CK(hipHostRegister(out + 16, n, hipHostRegisterMapped));
            CK(hipHostGetDevicePointer(&dout, out + 16, 0));
            (void)din;
            CK(hipMemcpyAsync(d_in, in + 16, n, hipMemcpyHostToDevice, s));
            kcopy(d_in, dout, n, s, 1024);
            CK(hipStreamSynchronize(s));
            CK(hipHostUnregister(out + 16));
            CK(hipHostUnregister(in + 16));
        });
        if (memcmp(out + 16, in + 16, n) != 0) {
            fprintf(stderr, "chain mismatch at %zu\n", n);
            return 1;
        }
        const double chain_pg = med([&] {
            CK(hipMemcpyAsync(d_in, in + 16, n, hipMemcpyHostToDevice, s));
            kcopy(d_in, d_out, n, s, 1024);
            CK(hipMemcpyAsync(out + 16, d_out, n, hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
        });
        printf("%8zu %6.1f %6.1f %6.1f %8.1f %8.1f %8.1f %7.1f %7.1f %8.1f\n", n, tr, tu, tru, h2d, kreg, kpin, rdm, chain,
               chain_pg);
        fflush(stdout);
    }
    return 0;
}
