// Unaligned global store probe (gfx950): do buffer_store_dwordx4 at byte offsets that are not
// multiples of 16 (or 4) write exactly their 16 bytes, and what bandwidth does a stream of them
// reach?  Each wave writes a contiguous 64 KiB region as 64-lane rows of 16-byte pieces starting
// at byte offset `mis` (so every store straddles two 16-byte segments when mis % 16 != 0), like a
// decode that stores each lane's 16 output bytes at an arbitrary output offset.
// build: hipcc --offload-arch=gfx950 -O3 tools/probes/unaligned_store_probe.hip -o build/unaligned_store_probe
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

__global__ __launch_bounds__(256) void writer(uint8_t* out, u32 region, u32 mis, u32 rows) {
    const u32 lane = threadIdx.x & 63;
    const u32 w = (u32)__builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + (threadIdx.x >> 6)));
    const u32x4 r = rsrc(out + (uint64_t)w * region, region);
    asm volatile("s_nop 4" ::: "memory");
    for (u32 k = 0; k < rows; ++k) {
        const u32 off = mis + 1024u * k + 16u * lane;
        u32x4 v;
        // byte j of the piece = (off + j) * 7 + w (a pattern the host can check)
        u32 b[16];
        for (u32 j = 0; j < 16; ++j) b[j] = ((off + j) * 7u + w) & 0xFFu;
        v.x = b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24);
        v.y = b[4] | (b[5] << 8) | (b[6] << 16) | (b[7] << 24);
        v.z = b[8] | (b[9] << 8) | (b[10] << 16) | (b[11] << 24);
        v.w = b[12] | (b[13] << 8) | (b[14] << 16) | (b[15] << 24);
        asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen" ::"v"(v), "v"(off), "s"(r) : "memory");
    }
}

int main() {
    const u32 region = 65536 + 64, rows = 63, waves = 16384;
    const size_t bytes = (size_t)region * waves;
    uint8_t* d;
    hipMalloc(&d, bytes);
    std::vector<uint8_t> h(region * 4);
    for (u32 mis : {0u, 1u, 4u, 8u, 13u}) {
        hipMemset(d, 0xEE, bytes);
        hipLaunchKernelGGL(writer, dim3(waves / 4), dim3(256), 0, 0, d, region, mis, rows);
        hipDeviceSynchronize();
        // check the first 4 waves' regions byte by byte
        hipMemcpy(h.data(), d, h.size(), hipMemcpyDeviceToHost);
        u32 bad = 0;
        for (u32 w = 0; w < 4; ++w)
            for (u32 p = 0; p < region; ++p) {
                const bool in = p >= mis && p < mis + 1024u * rows;
                const uint8_t want = in ? (uint8_t)((p * 7u + w) & 0xFFu) : 0xEE;
                if (h[(size_t)w * region + p] != want) ++bad;
            }
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        hipEventRecord(a, 0);
        for (int it = 0; it < 10; ++it)
            hipLaunchKernelGGL(writer, dim3(waves / 4), dim3(256), 0, 0, d, region, mis, rows);
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        const double gb = (double)waves * rows * 1024.0 * 10 / 1e9;
        printf("mis %2u: %s (%u bad bytes), %.1f us per launch, %.2f TB/s written\n", mis, bad ? "MISMATCH" : "byte-exact",
               bad, ms * 100.0, gb / (ms * 1e-3) / 1e3);
    }
    hipFree(d);
    return 0;
}
