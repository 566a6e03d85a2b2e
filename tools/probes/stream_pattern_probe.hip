// Access-pattern ceiling of the one-wave-per-buffer decode (decode_kernel on 16384 x 64 KiB): each
// wave owns one buffer, reads it in 1 KiB LDS-DMA tiles (kDepth slots, as walk_tiles / walk_ring),
// reads each tile back from LDS and stores kOut KiB per tile to its own output region (1 KiB per
// random / runs50 tile, 3 KiB per zero-filled tile), 4 waves per workgroup, LDS padded to set the
// waves per CU.  Against it: the same bytes copied grid-strided (every wave at adjacent addresses).
// Prints TB/s of (read + written) bytes.  No codec work: the memory pattern alone.
// build: hipcc --offload-arch=gfx950 -O3 tools/probes/stream_pattern_probe.hip -o build/stream_pattern_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

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
__device__ __forceinline__ u32 lds_addr(const void* p) {
    return (u32)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ void dma(u32x4 rs, u32 voff, u32 lds) {
    u32 keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_waitcnt lgkmcnt(0)\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(lds), "s"(rs) : "memory");
}
__device__ __forceinline__ void st16(u32x4 rs, u32 voff, u32x4 v) {
    asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen" ::"v"(v), "v"(voff), "s"(rs) : "memory");
}
#define VMW(N) case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
__device__ __forceinline__ void vmw(u32 n) {
    n = (u32)__builtin_amdgcn_readfirstlane((int)n);
    switch (n < 30u ? n : 30u) {
        VMW(0) VMW(1) VMW(2) VMW(3) VMW(4) VMW(5) VMW(6) VMW(7) VMW(8) VMW(9) VMW(10) VMW(11) VMW(12) VMW(13)
        VMW(14) VMW(15) VMW(16) VMW(17) VMW(18) VMW(19) VMW(20) VMW(21) VMW(22) VMW(23) VMW(24) VMW(25)
        VMW(26) VMW(27) VMW(28) VMW(29) VMW(30)
        default: break;
    }
}

// in: nbuf regions of inb bytes; out: nbuf regions of inb * kOut bytes.  kPad: extra LDS bytes per
// workgroup (occupancy).
template <u32 kOut, u32 kDepth, u32 kPad>
__global__ __launch_bounds__(256) void per_wave(const uint8_t* in, uint8_t* out, u32 nbuf, u32 inb) {
    __shared__ __attribute__((aligned(16))) uint8_t slots[4 * kDepth * 1024 + kPad];
    const u32 lane = threadIdx.x & 63, wid = (u32)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const u32 b = blockIdx.x * 4 + wid;
    if (kPad && threadIdx.x == 0) ((volatile uint8_t*)slots)[4 * kDepth * 1024] = 0;
    if (b >= nbuf) return;
    const u32x4 ri = rsrc(in + (uint64_t)b * inb, inb);
    const u32x4 ro = rsrc(out + (uint64_t)b * inb * kOut, inb * kOut);
    uint8_t* my = slots + wid * kDepth * 1024;
    const u32 l0 = (u32)__builtin_amdgcn_readfirstlane((int)lds_addr(my));
    const u32 nt = inb / 1024u;
    asm volatile("s_nop 4" ::: "memory");
    for (u32 d = 0; d < kDepth && d < nt; ++d) dma(ri, 1024u * d + 16u * lane, l0 + 1024u * d);
    for (u32 t = 0; t < nt; ++t) {
        // ops issued after tile t's load: the later priming loads and every earlier step's refill
        // and stores (t < D), else the stores of step t - D (which loaded tile t) and, for each step
        // j in (t - D, t), its refill (if any) and its stores
        u32 after = 0;
        if (t < kDepth) {
            for (u32 k = t + 1u; k < kDepth; ++k) after += k < nt ? 1u : 0u;
            for (u32 j = 0; j < t; ++j) after += (j + kDepth < nt ? 1u : 0u) + kOut;
        } else {
            after += kOut;
            for (u32 j = t - kDepth + 1u; j < t; ++j) after += (j + kDepth < nt ? 1u : 0u) + kOut;
        }
        vmw(after);
        const u32 s = t % kDepth;
        const u32x4 v = *reinterpret_cast<const u32x4*>(my + s * 1024u + 16u * lane);
        if (t + kDepth < nt) dma(ri, 1024u * (t + kDepth) + 16u * lane, l0 + 1024u * s);
#pragma unroll
        for (u32 q = 0; q < kOut; ++q) st16(ro, 1024u * (kOut * t + q) + 16u * lane, v + q);
    }
}


// The same with kBurst consecutive 1 KiB tiles per step: a wave's loads reach the memory as
// kBurst-KiB contiguous bursts (and its stores as kOut * kBurst KiB).
template <u32 kOut, u32 kDepth, u32 kPad, u32 kBurst>
__global__ __launch_bounds__(256) void per_wave_burst(const uint8_t* in, uint8_t* out, u32 nbuf, u32 inb) {
    __shared__ __attribute__((aligned(16))) uint8_t slots[4 * kDepth * kBurst * 1024 + kPad];
    const u32 lane = threadIdx.x & 63, wid = (u32)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const u32 b = blockIdx.x * 4 + wid;
    if (kPad && threadIdx.x == 0) ((volatile uint8_t*)slots)[4 * kDepth * kBurst * 1024] = 0;
    if (b >= nbuf) return;
    const u32x4 ri = rsrc(in + (uint64_t)b * inb, inb);
    const u32x4 ro = rsrc(out + (uint64_t)b * inb * kOut, inb * kOut);
    uint8_t* my = slots + wid * kDepth * kBurst * 1024;
    const u32 l0 = (u32)__builtin_amdgcn_readfirstlane((int)lds_addr(my));
    const u32 nt = inb / (1024u * kBurst);   // steps
    constexpr u32 kSt = kBurst * 1024u;
    asm volatile("s_nop 4" ::: "memory");
    for (u32 d = 0; d < kDepth && d < nt; ++d)
        for (u32 q = 0; q < kBurst; ++q) dma(ri, kSt * d + 1024u * q + 16u * lane, l0 + kSt * d + 1024u * q);
    for (u32 t = 0; t < nt; ++t) {
        u32 after = 0;
        if (t < kDepth) {
            for (u32 k = t + 1u; k < kDepth; ++k) after += k < nt ? kBurst : 0u;
            for (u32 j = 0; j < t; ++j) after += (j + kDepth < nt ? kBurst : 0u) + kOut * kBurst;
        } else {
            after += kOut * kBurst;
            for (u32 j = t - kDepth + 1u; j < t; ++j) after += (j + kDepth < nt ? kBurst : 0u) + kOut * kBurst;
        }
        vmw(after);
        const u32 s = t % kDepth;
        u32x4 v[kBurst];
#pragma unroll
        for (u32 q = 0; q < kBurst; ++q) v[q] = *reinterpret_cast<const u32x4*>(my + s * kSt + 1024u * q + 16u * lane);
        if (t + kDepth < nt)
            for (u32 q = 0; q < kBurst; ++q) dma(ri, kSt * (t + kDepth) + 1024u * q + 16u * lane, l0 + kSt * s + 1024u * q);
#pragma unroll
        for (u32 q = 0; q < kBurst; ++q)
#pragma unroll
            for (u32 o = 0; o < kOut; ++o) st16(ro, kOut * kSt * t + 1024u * (kOut * q + o) + 16u * lane, v[q] + o);
    }
}

__global__ void strided(u32x4* dst, const u32x4* src, uint64_t n16, uint64_t m16) {
    const uint64_t stride = (uint64_t)gridDim.x * 1024u;
    for (uint64_t base = (uint64_t)blockIdx.x * 1024u + threadIdx.x; base < n16; base += stride) {
        u32x4 v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint64_t i = base + 256u * q;
            if (i < n16) v[q] = src[i];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint64_t i = base + 256u * q;
            if (i < n16)
                for (uint64_t r = 0; r < m16 / n16; ++r) dst[i + r * n16] = v[q];
        }
    }
}

template <class F>
static float timeit(F f, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    f();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a, 0);
    for (int r = 0; r < reps; ++r) f();
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

template <u32 kOut, u32 kDepth, u32 kPad>
static void run(const char* name, const uint8_t* in, uint8_t* out, u32 nbuf, u32 inb) {
    const float ms = timeit([&] { hipLaunchKernelGGL((per_wave<kOut, kDepth, kPad>), dim3((nbuf + 3) / 4), dim3(256), 0, 0, in, out, nbuf, inb); }, 10);
    const double bytes = (double)nbuf * inb * (1 + kOut);
    printf("%-34s out/in %u depth %u pad %6u: %8.1f us  %.2f TB/s\n", name, kOut, kDepth, kPad, ms * 1e3, bytes / ms / 1e9);
}


template <u32 kOut, u32 kDepth, u32 kPad, u32 kBurst>
static void runb(const char* name, const uint8_t* in, uint8_t* out, u32 nbuf, u32 inb) {
    const float ms = timeit([&] { hipLaunchKernelGGL((per_wave_burst<kOut, kDepth, kPad, kBurst>), dim3((nbuf + 3) / 4), dim3(256), 0, 0, in, out, nbuf, inb); }, 10);
    const double bytes = (double)nbuf * inb * (1 + kOut);
    printf("%-34s out/in %u depth %u burst %u pad %6u: %8.1f us  %.2f TB/s\n", name, kOut, kDepth, kBurst, kPad, ms * 1e3, bytes / ms / 1e9);
}

int main() {
    const u32 nbuf = 16384, inb = 65536;
    uint8_t *in, *out;
    (void)hipMalloc(&in, (size_t)nbuf * inb);
    (void)hipMalloc(&out, (size_t)nbuf * inb * 3);
    (void)hipMemset(in, 1, (size_t)nbuf * inb);
    (void)hipMemset(out, 0, (size_t)nbuf * inb * 3);
    // (LDS per workgroup: 4 waves x depth KiB + pad; decode_kernel<96> holds ~22.6 KB: 7 per CU)
    run<1, 2, 0>("per-wave 1:1 (16 WG/CU cap)", in, out, nbuf, inb);
    run<1, 2, 14000>("per-wave 1:1 (~7 WG/CU)", in, out, nbuf, inb);
    run<1, 4, 6000>("per-wave 1:1 depth 4 (~7 WG/CU)", in, out, nbuf, inb);
    run<1, 2, 30000>("per-wave 1:1 (~4 WG/CU)", in, out, nbuf, inb);
    run<3, 2, 0>("per-wave 1:3 (16 WG/CU cap)", in, out, nbuf, inb / 3 / 1024 * 1024);
    run<3, 2, 14000>("per-wave 1:3 (~7 WG/CU)", in, out, nbuf, inb / 3 / 1024 * 1024);
    run<3, 4, 6000>("per-wave 1:3 depth 4 (~7 WG/CU)", in, out, nbuf, inb / 3 / 1024 * 1024);
    runb<1, 2, 6000, 2>("burst 2 KiB 1:1 (~7 WG/CU)", in, out, nbuf, inb);
    runb<1, 2, 0, 4>("burst 4 KiB 1:1 (~5 WG/CU)", in, out, nbuf, inb);
    runb<1, 2, 0, 2>("burst 2 KiB 1:1 (~10 WG/CU)", in, out, nbuf, inb);
    runb<3, 2, 2000, 2>("burst 2 KiB 1:3 (~7 WG/CU)", in, out, nbuf, inb / 3 / 2048 * 2048);
    {
        const uint64_t n16 = (uint64_t)nbuf * inb / 16;
        const float ms = timeit([&] { hipLaunchKernelGGL(strided, dim3(4096), dim3(256), 0, 0, (u32x4*)out, (const u32x4*)in, n16, n16); }, 10);
        printf("%-34s: %8.1f us  %.2f TB/s\n", "grid-strided copy 1:1", ms * 1e3, 2.0 * n16 * 16 / ms / 1e9);
        const uint64_t m = n16 / 3;
        const float ms3 = timeit([&] { hipLaunchKernelGGL(strided, dim3(4096), dim3(256), 0, 0, (u32x4*)out, (const u32x4*)in, m, 3 * m); }, 10);
        printf("%-34s: %8.1f us  %.2f TB/s\n", "grid-strided copy 1:3", ms3 * 1e3, 4.0 * m * 16 / ms3 / 1e9);
    }
    return 0;
}
