// Write-path probe: the codec's store pattern in isolation.  Each wave owns a contiguous region
// and writes it in 1 KiB wave-instructions (buffer_store_dwordx4, 16 B per lane, as dec_flush /
// the encode flush do), optionally with one 1 KiB LDS-DMA load per store (the tile pipeline's
// read side), optionally offset by 16 B from 128-B alignment, optionally with the nt bit.
// build: hipcc --offload-arch=gfx950 -O3 tools/probes/store_probe.hip -o build/store_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

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

template <int kMode>   // bit0: nt stores, bit1: LDS-DMA load per store, bit2: s_waitcnt per store
__global__ __launch_bounds__(256) void probe(uint8_t* out, const uint8_t* in, u32 region, u32 shift) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[4 * 1024];
    const u32 lane = threadIdx.x & 63, wid = (u32)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint64_t w = (uint64_t)blockIdx.x * 4 + wid;
    const u32x4 ro = rsrc(out + w * (region + 128) + shift, region);
    const u32x4 ri = rsrc(in + w * (region + 128), region);
    const u32 l0 = (u32)(uintptr_t)(const __attribute__((address_space(3))) void*)(lds + wid * 1024);
    u32x4 v = {lane, (u32)w, 0x55u, 0xAAu};
    asm volatile("s_nop 4" ::: "memory");
    for (u32 off = 0; off < region; off += 1024) {
        const u32 vo = off + 16 * lane;
        if (kMode & 2) {
            u32 keep;
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
                         : "=&s"(keep) : "v"(vo), "s"(l0), "s"(ri) : "memory");
        }
        if (kMode & 1)
            asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen nt" ::"v"(v), "v"(vo), "s"(ro) : "memory");
        else
            asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen" ::"v"(v), "v"(vo), "s"(ro) : "memory");
        if (kMode & 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        v.z += 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int kMode>
float run(uint8_t* out, const uint8_t* in, u32 waves, u32 region, u32 shift) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(probe<kMode>, dim3(waves / 4), dim3(256), 0, 0, out, in, region, shift);
    (void)hipEventRecord(a, 0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(probe<kMode>, dim3(waves / 4), dim3(256), 0, 0, out, in, region, shift);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / 5;
}

int main() {
    const u32 region = 64 * 1024, waves = 16384;
    const size_t bytes = (size_t)waves * (region + 128) + 4096;
    uint8_t *out, *in;
    if (hipMalloc(&out, bytes) != hipSuccess || hipMalloc(&in, bytes) != hipSuccess) return 1;
    (void)hipMemset(in, 1, bytes);
    const double wb = (double)waves * region;
    for (u32 shift : {0u, 16u}) {
        float t0 = run<0>(out, in, waves, region, shift), t1 = run<1>(out, in, waves, region, shift);
        float t2 = run<2>(out, in, waves, region, shift), t3 = run<3>(out, in, waves, region, shift);
        float t6 = run<6>(out, in, waves, region, shift);
        printf("shift %2u: store %.0f GB/s | nt %.0f GB/s | +lds-dma load (r+w) %.0f GB/s | nt+load %.0f GB/s | load+vmcnt(8) %.0f GB/s\n",
               shift, wb / t0 / 1e6, wb / t1 / 1e6, 2 * wb / t2 / 1e6, 2 * wb / t3 / 1e6, 2 * wb / t6 / 1e6);
    }
    return 0;
}
