// Host path: what registering the server's buffers would cost against the drop-in's
// pinned staging.  The reference server allocates a request's payload per request
// (/root/reference/src/server.c:150-151, calloc + readn) and its response per request (:262-266), so a
// registration would be per call.  Per size: hipHostRegister + hipHostUnregister of a fresh calloc'd
// buffer; a memcpy into a long-lived pinned staging buffer (the library's path); host-to-device copies
// from pinned, registered and pageable memory.  Medians of 25 reps, microseconds.
// build: hipcc -O2 tools/probes/host_register_probe.cpp -o build/host_register_probe
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
static double med(F f, int reps = 25) {
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

int main() {
    const size_t kMax = 4u << 20;
    void *pinned, *dev;
    CK(hipHostMalloc(&pinned, kMax, hipHostMallocDefault));
    CK(hipMalloc(&dev, kMax));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    printf("%10s %14s %12s %12s %12s %12s\n", "bytes", "reg+unreg", "memcpy->pin", "H2D pinned", "H2D reg", "H2D pageable");
    for (size_t n : {4096ul, 16384ul, 65536ul, 262144ul, 1048576ul, 4194304ul}) {
        // a fresh request buffer each time, as the server's calloc per request
        const double reg = med([&] {
            char* p = (char*)calloc(n, 1);
            p[0] = 1;
            CK(hipHostRegister(p, n, hipHostRegisterDefault));
            CK(hipHostUnregister(p));
            free(p);
        });
        char* src = (char*)calloc(n, 1);
        memset(src, 7, n);
        const double cp = med([&] { memcpy(pinned, src, n); });
        const double h2d_pin = med([&] {
            CK(hipMemcpyAsync(dev, pinned, n, hipMemcpyHostToDevice, s));
            CK(hipStreamSynchronize(s));
        });
        CK(hipHostRegister(src, n, hipHostRegisterDefault));
        const double h2d_reg = med([&] {
            CK(hipMemcpyAsync(dev, src, n, hipMemcpyHostToDevice, s));
            CK(hipStreamSynchronize(s));
        });
        CK(hipHostUnregister(src));
        const double h2d_page = med([&] {
            CK(hipMemcpyAsync(dev, src, n, hipMemcpyHostToDevice, s));
            CK(hipStreamSynchronize(s));
        });
        free(src);
        printf("%10zu %14.1f %12.1f %12.1f %12.1f %12.1f\n", n, reg, cp, h2d_pin, h2d_reg, h2d_page);
    }
    return 0;
}
