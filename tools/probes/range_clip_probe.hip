// Buffer range-check probe (gfx950): what does a buffer_store_dwordx4 that straddles num_records
// write?  One wave; lane l stores 16 pattern bytes at byte offset 16 l + mis into a buffer whose
// descriptor range is N bytes; the host reports, per (mis, N), whether exactly the in-range bytes
// [0, N) landed (per-byte clipping), whole dwords were dropped, or the whole store was dropped.
// build: hipcc --offload-arch=gfx950 -O3 tools/probes/range_clip_probe.hip -o build/range_clip_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>

typedef uint32_t u32;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 rsrc(const void* base, u32 n) {
    const uint64_t a = (uint64_t)base;
    u32x4 r;
    r.x = (u32)a;
    r.y = (u32)(a >> 32) & 0xFFFFu;
    r.z = n;
    r.w = 0x00020000u;
    return r;
}

__global__ void writer(uint8_t* out, u32 n, u32 mis) {
    const u32 lane = threadIdx.x;
    const u32x4 r = rsrc(out, n);
    asm volatile("s_nop 4" ::: "memory");
    const u32 off = 16u * lane + mis;
    u32 b[16];
    for (u32 j = 0; j < 16; ++j) b[j] = (off + j + 1u) & 0xFFu;   // (positions whose pattern byte is 0xEE are not judged)
    u32x4 v;
    v.x = b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24);
    v.y = b[4] | (b[5] << 8) | (b[6] << 16) | (b[7] << 24);
    v.z = b[8] | (b[9] << 8) | (b[10] << 16) | (b[11] << 24);
    v.w = b[12] | (b[13] << 8) | (b[14] << 16) | (b[15] << 24);
    asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen" ::"v"(v), "v"(off), "s"(r) : "memory");
}

int main() {
    const u32 cap = 2048;
    uint8_t* d;
    hipMalloc(&d, cap);
    std::vector<uint8_t> h(cap);
    u32 exact = 0, cases = 0;
    for (u32 n : {100u, 101u, 102u, 103u, 104u, 111u, 112u, 113u, 1000u}) {
        for (u32 mis = 0; mis < 16; ++mis) {
            hipMemset(d, 0xEE, cap);
            hipLaunchKernelGGL(writer, dim3(1), dim3(64), 0, 0, d, n, mis);
            hipDeviceSynchronize();
            hipMemcpy(h.data(), d, cap, hipMemcpyDeviceToHost);
            // expected under per-byte clipping: bytes [mis, min(n, 1024 + mis)) written
            u32 hi_written = 0, missing = 0, extra = 0;
            for (u32 p = 0; p < cap; ++p) {
                const bool w = h[p] == (uint8_t)((p + 1u) & 0xFFu) && h[p] != 0xEE;
                const bool want = p >= mis && p < n && p < 1024u + mis;
                if (w) hi_written = p + 1;
                if (want && !w && ((p + 1u) & 0xFFu) != 0xEE) ++missing;
                if (!want && w) ++extra;
            }
            ++cases;
            if (!missing && !extra) ++exact;
            printf("N %4u mis %2u: written up to %4u, missing %u, past-range %u\n", n, mis, hi_written, missing, extra);
        }
    }
    printf("%u of %u cases clip exactly at N\n", exact, cases);
    hipFree(d);
    return 0;
}
