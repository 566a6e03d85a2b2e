// Host path of large calls: where a 1 MiB drop-in call's time
// goes, and which transfer form moves the caller's bytes to the device and the result back fastest.
// Per size, medians of 40 reps in microseconds, one stream:
//   memcpy     caller buffer -> long-lived pinned buffer (the staged path's host copy)
//   sdma_h2d   hipMemcpyAsync pinned -> device + sync     sdma_d2h  device -> pinned + sync
//   page_h2d   hipMemcpyAsync pageable -> device + sync   page_d2h  device -> pageable + sync
//   kern_h2d   a copy kernel reading the mapped pinned buffer into device memory + sync
//   kern_d2h   a copy kernel writing device memory into the mapped pinned buffer + sync
//   chain_*    a whole call's transfers and one device pass (d_in -> d_out copy on the device):
//     page     pageable H2D, device pass, pageable D2H (the library's direct staging)
//     sdma     memcpy in, pinned H2D, device pass, pinned D2H, memcpy out
//     kern     memcpy in, copy kernel in, device pass, copy kernel out, memcpy out (one sync)
//     pipe     as sdma with the memcpys in 4 chunks overlapping the DMAs (events per chunk)
//     kpipe    as kern, the memcpy in chunks overlapping per-chunk copy kernels, memcpy out
//              per chunk behind per-chunk copy kernels (events)
// build: hipcc -O2 --offload-arch=gfx950 tools/probes/hostpath_pipe_probe.hip -o build/hostpath_pipe_probe
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

// n16 16-byte words, grid-stride
__global__ void __launch_bounds__(256) copy16(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        const uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
        dst[i] = a; dst[i + stride] = b; dst[i + 2 * stride] = c; dst[i + 3 * stride] = d;
    }
    for (; i < n16; i += stride) dst[i] = src[i];
}

static void kcopy(const void* s, void* d, size_t n, hipStream_t st, int grid) {
    const size_t n16 = n / 16;
    int g = grid;
    const size_t need = (n16 + 255) / 256;
    if ((size_t)g > need) g = (int)need;
    hipLaunchKernelGGL(copy16, dim3(g), dim3(256), 0, st, (const uint4*)s, (uint4*)d, n16);
}

int main() {
    const size_t kMax = 4u << 20;
    const int kCh = 4;
    uint8_t *h_in, *h_out, *d_in, *d_out, *dh_in, *dh_out;
    CK(hipHostMalloc(&h_in, kMax, hipHostMallocMapped));
    CK(hipHostMalloc(&h_out, kMax, hipHostMallocMapped));
    CK(hipHostGetDevicePointer((void**)&dh_in, h_in, 0));
    CK(hipHostGetDevicePointer((void**)&dh_out, h_out, 0));
    CK(hipMalloc(&d_in, kMax));
    CK(hipMalloc(&d_out, kMax));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t ev[kCh];
    for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    std::vector<uint8_t> src(kMax), dst(kMax);
    for (size_t i = 0; i < kMax; ++i) src[i] = (uint8_t)((i * 2654435761u) >> 13);
    printf("%8s %7s %8s %8s %8s %8s %8s %8s %8s %8s %8s %8s %8s %8s\n", "bytes", "memcpy", "sdma_h2d", "sdma_d2h",
           "page_h2d", "page_d2h", "kern_h2d", "kern_d2h", "kh2d_1k", "c_page", "c_sdma", "c_kern", "c_pipe", "c_kpipe");
    for (size_t n : {262144ul, 1048576ul, 4194304ul}) {
        const double cp = med([&] { memcpy(h_in, src.data(), n); });
        const double sh = med([&] { CK(hipMemcpyAsync(d_in, h_in, n, hipMemcpyHostToDevice, s)); CK(hipStreamSynchronize(s)); });
        const double sd = med([&] { CK(hipMemcpyAsync(h_out, d_out, n, hipMemcpyDeviceToHost, s)); CK(hipStreamSynchronize(s)); });
        const double ph = med([&] { CK(hipMemcpyAsync(d_in, src.data(), n, hipMemcpyHostToDevice, s)); CK(hipStreamSynchronize(s)); });
        const double pd = med([&] { CK(hipMemcpyAsync(dst.data(), d_out, n, hipMemcpyDeviceToHost, s)); CK(hipStreamSynchronize(s)); });
        const double kh = med([&] { kcopy(dh_in, d_in, n, s, 256); CK(hipStreamSynchronize(s)); });
        const double kd = med([&] { kcopy(d_out, dh_out, n, s, 256); CK(hipStreamSynchronize(s)); });
        const double kh1 = med([&] { kcopy(dh_in, d_in, n, s, 1024); CK(hipStreamSynchronize(s)); });
        const double c_page = med([&] {
            CK(hipMemcpyAsync(d_in, src.data(), n, hipMemcpyHostToDevice, s));
            kcopy(d_in, d_out, n, s, 1024);
            CK(hipMemcpyAsync(dst.data(), d_out, n, hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
        });
        const double c_sdma = med([&] {
            memcpy(h_in, src.data(), n);
            CK(hipMemcpyAsync(d_in, h_in, n, hipMemcpyHostToDevice, s));
            kcopy(d_in, d_out, n, s, 1024);
            CK(hipMemcpyAsync(h_out, d_out, n, hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
            memcpy(dst.data(), h_out, n);
        });
        const double c_kern = med([&] {
            memcpy(h_in, src.data(), n);
            kcopy(dh_in, d_in, n, s, 256);
            kcopy(d_in, d_out, n, s, 1024);
            kcopy(d_out, dh_out, n, s, 256);
            CK(hipStreamSynchronize(s));
            memcpy(dst.data(), h_out, n);
        });
        const size_t ch = n / kCh;
        const double c_pipe = med([&] {
            for (int k = 0; k < kCh; ++k) {
                memcpy(h_in + k * ch, src.data() + k * ch, ch);
                CK(hipMemcpyAsync(d_in + k * ch, h_in + k * ch, ch, hipMemcpyHostToDevice, s));
            }
            kcopy(d_in, d_out, n, s, 1024);
            for (int k = 0; k < kCh; ++k) {
                CK(hipMemcpyAsync(h_out + k * ch, d_out + k * ch, ch, hipMemcpyDeviceToHost, s));
                CK(hipEventRecord(ev[k], s));
            }
            for (int k = 0; k < kCh; ++k) {
                CK(hipEventSynchronize(ev[k]));
                memcpy(dst.data() + k * ch, h_out + k * ch, ch);
            }
        });
        const double c_kpipe = med([&] {
            for (int k = 0; k < kCh; ++k) {
                memcpy(h_in + k * ch, src.data() + k * ch, ch);
                kcopy(dh_in + k * ch, d_in + k * ch, ch, s, 256);
            }
            kcopy(d_in, d_out, n, s, 1024);
            for (int k = 0; k < kCh; ++k) {
                kcopy(d_out + k * ch, dh_out + k * ch, ch, s, 256);
                CK(hipEventRecord(ev[k], s));
            }
            for (int k = 0; k < kCh; ++k) {
                CK(hipEventSynchronize(ev[k]));
                memcpy(dst.data() + k * ch, h_out + k * ch, ch);
            }
        });
        if (memcmp(dst.data(), src.data(), n) != 0) {
            fprintf(stderr, "round trip mismatch at %zu bytes\n", n);
            return 1;
        }
        printf("%8zu %7.1f %8.1f %8.1f %8.1f %8.1f %8.1f %8.1f %8.1f %8.1f %8.1f %8.1f %8.1f %8.1f\n", n, cp, sh, sd, ph,
               pd, kh, kd, kh1, c_page, c_sdma, c_kern, c_pipe, c_kpipe);
        fflush(stdout);
    }
    return 0;
}
