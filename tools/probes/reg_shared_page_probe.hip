// Two host registrations that share a page (csrc/rle_dropin.cpp LargeCall, round 6): a read-only
// one (the call's input, hipHostRegisterReadOnly) and a read-write one right after it (the result
// block, malloc'd next to it on the heap).  A kernel writes every byte of the read-write range
// through its device address; the host then checks them, the shared page's bytes in particular.
// Cases: read-only first then read-write, the reverse order, both read-write, one registration of
// the union.   build: hipcc -O2 --offload-arch=gfx950 tools/probes/reg_shared_page_probe.hip -o build/reg_shared_page_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                     \
            return -1;                                                                  \
        }                                                                               \
    } while (0)

__global__ void fill(uint8_t* dst, size_t n, uint8_t v) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = (uint8_t)(v + i);
}

// returns the number of wrong bytes (and of them, those in the page shared with the input)
static long run(int mode, size_t in_n, size_t out_n, size_t gap, long* shared_bad) {
    const size_t page = 4096, total = in_n + gap + out_n + 2 * page;
    uint8_t* base = (uint8_t*)aligned_alloc(page, (total + page - 1) / page * page);
    memset(base, 0x5a, total);
    uint8_t* in = base + 100;                 // not page aligned, like a heap block
    uint8_t* out = in + in_n + gap;          // right after it: shares in's last page
    void *d_out = nullptr, *d_u = nullptr;
    hipStream_t s;
    CK(hipStreamCreate(&s));
    if (mode == 0 || mode == 2) {   // input first (read-only / read-write), then the result block
        CK(hipHostRegister(in, in_n, hipHostRegisterMapped | (mode == 0 ? hipHostRegisterReadOnly : 0u)));
        CK(hipHostRegister(out, out_n, hipHostRegisterMapped));
        CK(hipHostGetDevicePointer(&d_out, out, 0));
    } else if (mode == 1) {         // the result block first, then the input read-only
        CK(hipHostRegister(out, out_n, hipHostRegisterMapped));
        CK(hipHostRegister(in, in_n, hipHostRegisterMapped | hipHostRegisterReadOnly));
        CK(hipHostGetDevicePointer(&d_out, out, 0));
    } else {                        // one registration of the union
        CK(hipHostRegister(in, in_n + gap + out_n, hipHostRegisterMapped));
        CK(hipHostGetDevicePointer(&d_u, in, 0));
        d_out = (uint8_t*)d_u + in_n + gap;
    }
    hipLaunchKernelGGL(fill, dim3(256), dim3(256), 0, s, (uint8_t*)d_out, out_n, (uint8_t)mode);
    CK(hipStreamSynchronize(s));
    long bad = 0, sbad = 0;
    const uintptr_t shared_end = (((uintptr_t)in + in_n + page - 1) / page) * page;
    for (size_t i = 0; i < out_n; ++i)
        if (out[i] != (uint8_t)(mode + i)) {
            ++bad;
            if ((uintptr_t)(out + i) < shared_end) ++sbad;
        }
    if (mode == 3) {
        CK(hipHostUnregister(in));
    } else {
        CK(hipHostUnregister(out));
        CK(hipHostUnregister(in));
    }
    CK(hipStreamDestroy(s));
    free(base);
    *shared_bad = sbad;
    return bad;
}

int main() {
    const char* names[] = {"ro input first", "rw result first", "both rw", "union"};
    int fails = 0;
    for (int rep = 0; rep < 3; ++rep)
        for (int mode = 0; mode < 4; ++mode)
            for (size_t in_n : {262165ul, 1052732ul})
                for (size_t gap : {0ul, 16ul, 1000ul}) {
                    long sb = 0;
                    const long bad = run(mode, in_n, 393216, gap, &sb);
                    if (bad) ++fails;
                    printf("%-16s in=%zu gap=%zu: wrong bytes %ld (in the shared page %ld)\n", names[mode], in_n, gap,
                           bad, sb);
                }
    printf("cases with wrong bytes: %d\n", fails);
    return fails ? 1 : 0;
}
