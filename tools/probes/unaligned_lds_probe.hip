// Unaligned LDS access probe (gfx950): do ds_write_b32 / ds_write_b64 / ds_read_b32 / ds_read_b64 at
// byte addresses that are not multiples of their width give the bytes a byte-wise model gives, and
// what do they cost?  Each wave: zero 4 KiB of LDS, every lane writes a pattern at 4 KiB-bounded
// random byte offsets (non-overlapping per lane), read back as bytes and compare.
// build: hipcc --offload-arch=gfx950 -O3 tools/probes/unaligned_lds_probe.hip -o build/unaligned_lds_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ unsigned lds_addr(const void* p) {
    return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

__global__ void check(unsigned* err, unsigned* got) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[4096];
    const unsigned lane = threadIdx.x;
    for (unsigned k = lane; k < 1024; k += 64) reinterpret_cast<unsigned*>(buf)[k] = 0;
    __syncthreads();
    // lane l writes at 64*l + (l % 8) (distinct 64-byte slots, all misalignments 0..7)
    const unsigned off = 64 * lane + (lane % 8);
    const unsigned a = lds_addr(buf) + off;
    const unsigned v32 = 0xA1B2C3D4u ^ lane;
    const uint64_t v64 = 0x1122334455667788ull ^ ((uint64_t)lane << 40);
    asm volatile("ds_write_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(a), "v"(v32) : "memory");
    asm volatile("ds_write_b64 %0, %1 offset:16\n\ts_waitcnt lgkmcnt(0)" ::"v"(a), "v"(v64) : "memory");
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v128 = {0x01020304u ^ lane, 0x05060708u, 0x090A0B0Cu, 0x0D0E0F10u ^ (lane << 8)};
    asm volatile("ds_write_b128 %0, %1 offset:32\n\ts_waitcnt lgkmcnt(0)" ::"v"(a), "v"(v128) : "memory");
    __syncthreads();
    unsigned e = 0;
    for (unsigned j = 0; j < 4; ++j)
        if (buf[off + j] != ((v32 >> (8 * j)) & 0xFF)) e |= 1;
    for (unsigned j = 0; j < 8; ++j)
        if (buf[off + 16 + j] != ((v64 >> (8 * j)) & 0xFF)) e |= 2;
    for (unsigned j = 0; j < 16; ++j)
        if (buf[off + 32 + j] != ((v128[j / 4] >> (8 * (j % 4))) & 0xFF)) e |= 64;
    if (buf[off + 31] != 0 || buf[off + 48] != 0) e |= 128;
    // neighbours untouched
    if (off > 0 && buf[off - 1] != 0) e |= 4;
    if (buf[off + 4] != 0 || buf[off + 24] != 0) e |= 8;
    unsigned r32;
    uint64_t r64;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r32) : "v"(a) : "memory");
    asm volatile("ds_read_b64 %0, %1 offset:16\n\ts_waitcnt lgkmcnt(0)" : "=v"(r64) : "v"(a) : "memory");
    if (r32 != v32) e |= 16;
    if (r64 != v64) e |= 32;
    got[lane] = r32;
    if (e) atomicOr(err, e | (1u << (8 + (lane % 8))));
}

template <int kW>
__global__ void timing(unsigned* sink, unsigned mis, int iters) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[16384];
    const unsigned lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    // lanes ~17 bytes apart (a random-data decode's spacing), + mis
    const unsigned base = lds_addr(buf) + wid * 4096 + 17 * lane * (kW == 8 ? 2 : 1) + mis;
    unsigned v = lane;
    uint64_t v2 = lane;
    for (int i = 0; i < iters; ++i) {
        const unsigned a = base + (i & 7);
        if (kW == 1) asm volatile("ds_write_b8 %0, %1" ::"v"(a), "v"(v) : "memory");
        if (kW == 2) asm volatile("ds_write_b16 %0, %1" ::"v"(a & ~1u), "v"(v) : "memory");
        if (kW == 4) asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(v) : "memory");
        if (kW == 5) asm volatile("ds_write_b32 %0, %1" ::"v"(a & ~3u), "v"(v) : "memory");
        if (kW == 8) asm volatile("ds_write_b64 %0, %1" ::"v"(a), "v"(v2) : "memory");
        if (kW == 9) asm volatile("ds_write_b64 %0, %1" ::"v"(a & ~7u), "v"(v2) : "memory");
        v += 1;
        v2 += 1;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) sink[blockIdx.x] = buf[5];
}

// the decode scatter's layout: lane l's 16 u16 keys at 32 l + 2 r + 2 (r = 0..15; +2: 2-byte
// misalignment of a random-data lane's output), written as 16 x ds_write_b16 (kW 16) or as two
// unaligned ds_write_b128 (kW 128)
template <int kW>
__global__ void scatter(unsigned* sink, int iters) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[4 * 8192];
    const unsigned lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    u32x4 v = {lane, lane + 1, lane + 2, lane + 3};
    for (int i = 0; i < iters; ++i) {
        const unsigned a = lds_addr(buf) + wid * 8192 + 32 * lane + 2 + ((i & 3) << 11);
        if (kW == 16) {
#pragma unroll
            for (int r = 0; r < 16; ++r) asm volatile("ds_write_b16 %0, %1 offset:%2" ::"v"(a), "v"(v.x), "i"(2 * r) : "memory");
        } else {
            asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(v) : "memory");
            asm volatile("ds_write_b128 %0, %1 offset:16" ::"v"(a), "v"(v) : "memory");
        }
        v.x += 1;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) sink[blockIdx.x] = buf[5];
}
template <int kW>
void time_scatter(const char* name, unsigned* sink) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int iters = 2048, blocks = 256 * 4;
    hipLaunchKernelGGL(scatter<kW>, dim3(blocks), dim3(256), 0, 0, sink, iters);
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL(scatter<kW>, dim3(blocks), dim3(256), 0, 0, sink, iters);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    // per CU: 4 blocks x 4 waves, each iteration = one lane-row of 32 key bytes per lane
    printf("%-40s %8.3f ms  %.1f cycles per wave-row of keys per CU (2.4 GHz)\n", name, ms,
           ms * 1e-3 * 2.4e9 * 256 / ((double)blocks * 4 * iters));
}

template <int kW>
void time_one(const char* name, unsigned* sink) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int iters = 4096, blocks = 256 * 8;
    hipLaunchKernelGGL(timing<kW>, dim3(blocks), dim3(256), 0, 0, sink, 1u, iters);
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL(timing<kW>, dim3(blocks), dim3(256), 0, 0, sink, 1u, iters);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    // wave-instructions per CU per cycle at 2.4 GHz (256 CUs)
    const double winst = (double)blocks * 4 * iters;
    printf("%-28s %8.3f ms  %.2f cycles per wave-instruction per CU (2.4 GHz)\n", name, ms,
           ms * 1e-3 * 2.4e9 * 256 / winst);
}

int main() {
    unsigned *err, *got, *sink;
    (void)hipMalloc(&err, 4);
    (void)hipMalloc(&got, 256);
    (void)hipMalloc(&sink, 1 << 20);
    (void)hipMemset(err, 0, 4);
    hipLaunchKernelGGL(check, dim3(1), dim3(64), 0, 0, err, got);
    unsigned h = 0;
    (void)hipMemcpy(&h, err, 4, hipMemcpyDeviceToHost);
    printf("unaligned check: err=0x%x (%s)\n", h, h ? "MISMATCH" : "byte-exact");
    time_one<1>("ds_write_b8 any", sink);
    time_one<2>("ds_write_b16 aligned", sink);
    time_one<5>("ds_write_b32 aligned", sink);
    time_one<4>("ds_write_b32 unaligned", sink);
    time_one<9>("ds_write_b64 aligned", sink);
    time_one<8>("ds_write_b64 unaligned", sink);
    time_scatter<16>("scatter 16 x ds_write_b16 (decode today)", sink);
    time_scatter<128>("scatter 2 x ds_write_b128 unaligned", sink);
    return 0;
}
