// Decode memory-pattern variants on a dec64k-shaped batch: 16384 buffers of
// 45 KiB in (the 1 KiB tiles a decode reads) and 64 KiB out, each tile writing its share of the
// buffer's output (shares on 128-byte lines, so split lines are not what is measured), no codec
// work.  The same bytes, four ways of giving tiles to waves:
//   A  one wave per buffer walking its tiles (decode_kernel's pattern), 4 waves per workgroup,
//      LDS padded to decode_kernel<96>'s 7 workgroups per CU
//   B  the 4 waves of a workgroup share one buffer, wave w taking tiles w, w + 4, ...
//   C  kW-wave workgroups per buffer in rounds of kW tiles with a barrier per round (a
//      cooperative decode's pattern)
//   D  arena order: a resident grid of waves, wave k taking global tiles k, k + W, k + 2W, ...
//      (all waves in flight sit in one contiguous window of the arena, as in a copy)
// plus the grid-strided copy of the same bytes.  Each tile: LDS-DMA into a 2-slot ring, read back,
// stores of its output share.  Prints time, TB/s of (in + out) bytes and the fraction of 8 TB/s.
// build: hipcc --offload-arch=gfx950 -O3 tools/probes/pattern_variants_probe.hip -o build/pattern_variants_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));

constexpr u32 kNbuf = 16384, kTiles = 45, kInB = kTiles * 1024u, kOutB = 65536u;

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
__device__ __forceinline__ u32 uni(u32 v) { return (u32)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ void dma(u32x4 rs, u32 voff, u32 lds) {
    u32 keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_waitcnt lgkmcnt(0)\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(lds), "s"(rs) : "memory");
}
__device__ __forceinline__ void st16(u32x4 rs, u32 voff, u32x4 v) {
    asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen" ::"v"(v), "v"(voff), "s"(rs) : "memory");
}
__device__ __forceinline__ void vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
#define VMW(N) case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
__device__ __forceinline__ void vmw(u32 n) {
    switch (uni(n) < 8u ? uni(n) : 8u) {
        VMW(0) VMW(1) VMW(2) VMW(3) VMW(4) VMW(5) VMW(6) VMW(7) VMW(8)
        default: break;
    }
}
// output share of tile t: [lo, hi) on 128-byte lines
__device__ __forceinline__ u32 share(u32 t) { return t >= kTiles ? kOutB : (u32)(((uint64_t)t * kOutB / kTiles) & ~127ull); }
// The stores of one tile (value v from the slot): ceil(share / 1 KiB) instructions, lanes past the
// share clipped by the range check.  Returns the instructions issued.
__device__ __forceinline__ u32 put(u32x4 ro, u32 t, u32 lane, u32x4 v) {
    const u32 lo = share(t), hi = share(t + 1u);
    const u32 n = (hi - lo + 1023u) / 1024u;
    for (u32 k = 0; k < n; ++k) {
        const u32 a = lo + 1024u * k + 16u * lane;
        st16(ro, a < hi ? a : 0x7FFFFFF0u, v);
    }
    return n;
}

// ---------------------------------------------------------------- A: one wave per buffer
template <u32 kPad>
__global__ __launch_bounds__(256) void pat_a(const uint8_t* in, uint8_t* out) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[4 * 2 * 1024 + kPad];
    const u32 lane = threadIdx.x & 63, wid = uni(threadIdx.x >> 6);
    if (kPad && threadIdx.x == 0) ((volatile uint8_t*)lds)[4 * 2048 + blockIdx.x % kPad] = 0;
    const u32 b = blockIdx.x * 4 + wid;
    if (b >= kNbuf) return;
    const u32x4 ri = rsrc(in + (uint64_t)b * kInB, kInB);
    const u32x4 ro = rsrc(out + (uint64_t)b * kOutB, kOutB);
    uint8_t* my = lds + wid * 2048;
    const u32 l0 = uni(lds_addr(my));
    asm volatile("s_nop 4" ::: "memory");
    dma(ri, 16u * lane, l0);
    dma(ri, 1024u + 16u * lane, l0 + 1024u);
    u32 prev_st = 0;   // stores issued after the tile now awaited
    for (u32 t = 0; t < kTiles; ++t) {
        // issued after tile t's load: (t == 0) tile 1's load; else the refill of step t-1 (which is
        // tile t+1) and step t-1's stores
        vmw(t == 0 ? 1u : (t + 1u < kTiles ? 1u : 0u) + prev_st);
        const u32 s = t & 1u;
        const u32x4 v = *reinterpret_cast<const u32x4*>(my + s * 1024u + 16u * lane);
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the slot is read before it is refilled
        if (t + 2u < kTiles) dma(ri, 1024u * (t + 2u) + 16u * lane, l0 + 1024u * s);
        prev_st = put(ro, t, lane, v);
    }
}

// ---------------------------------------------------------------- B: 4 waves share a buffer
template <u32 kPad>
__global__ __launch_bounds__(256) void pat_b(const uint8_t* in, uint8_t* out) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[4 * 2 * 1024 + kPad];
    const u32 lane = threadIdx.x & 63, wid = uni(threadIdx.x >> 6);
    if (kPad && threadIdx.x == 0) ((volatile uint8_t*)lds)[4 * 2048 + blockIdx.x % kPad] = 0;
    const u32 b = blockIdx.x;
    if (b >= kNbuf) return;
    const u32x4 ri = rsrc(in + (uint64_t)b * kInB, kInB);
    const u32x4 ro = rsrc(out + (uint64_t)b * kOutB, kOutB);
    uint8_t* my = lds + wid * 2048;
    const u32 l0 = uni(lds_addr(my));
    asm volatile("s_nop 4" ::: "memory");
    const u32 n = (kTiles - wid + 3u) / 4u;   // this wave's tiles: wid + 4 i
    if (n > 0) dma(ri, 1024u * wid + 16u * lane, l0);
    if (n > 1) dma(ri, 1024u * (wid + 4u) + 16u * lane, l0 + 1024u);
    u32 prev_st = 0;
    for (u32 i = 0; i < n; ++i) {
        vmw(i == 0 ? (n > 1 ? 1u : 0u) : (i + 1u < n ? 1u : 0u) + prev_st);
        const u32 s = i & 1u;
        const u32x4 v = *reinterpret_cast<const u32x4*>(my + s * 1024u + 16u * lane);
        __builtin_amdgcn_s_waitcnt(0xc07f);
        if (i + 2u < n) dma(ri, 1024u * (wid + 4u * (i + 2u)) + 16u * lane, l0 + 1024u * s);
        prev_st = put(ro, wid + 4u * i, lane, v);
    }
}

// ---------------------------------------------------------------- C: kW-wave rounds per buffer
template <u32 kW, u32 kPad>
__global__ __launch_bounds__(64 * kW) void pat_c(const uint8_t* in, uint8_t* out) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kW * 2 * 1024 + kPad];
    const u32 lane = threadIdx.x & 63, wid = uni(threadIdx.x >> 6);
    if (kPad && threadIdx.x == 0) ((volatile uint8_t*)lds)[kW * 2048 + blockIdx.x % kPad] = 0;
    const u32 b = blockIdx.x;
    if (b >= kNbuf) return;
    const u32x4 ri = rsrc(in + (uint64_t)b * kInB, kInB);
    const u32x4 ro = rsrc(out + (uint64_t)b * kOutB, kOutB);
    uint8_t* my = lds + wid * 2048;
    const u32 l0 = uni(lds_addr(my));
    asm volatile("s_nop 4" ::: "memory");
    const u32 rounds = (kTiles + kW - 1u) / kW;
    dma(ri, 1024u * wid + 16u * lane, l0);   // (past the buffer: clipped to zeros)
    u32 prev_st = 0;
    for (u32 r = 0; r < rounds; ++r) {
        const u32 t = r * kW + wid;
        if (r + 1u < rounds) dma(ri, 1024u * (t + kW) + 16u * lane, l0 + 1024u * ((r + 1u) & 1u));
        // this round's tile: issued before the last round's stores and this round's refill
        vmw((r + 1u < rounds ? 1u : 0u) + prev_st);
        __syncthreads();
        const u32x4 v = *reinterpret_cast<const u32x4*>(my + (r & 1u) * 1024u + 16u * lane);
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __syncthreads();   // (the cooperative decode's second exchange; the slot read before its refill)
        prev_st = t < kTiles ? put(ro, t, lane, v) : 0u;
    }
}

// ---------------------------------------------------------------- D: arena order, resident grid
template <u32 kPad>
__global__ __launch_bounds__(256) void pat_d(const uint8_t* in, uint8_t* out) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[4 * 2 * 1024 + kPad];
    const u32 lane = threadIdx.x & 63, wid = uni(threadIdx.x >> 6);
    if (kPad && threadIdx.x == 0) ((volatile uint8_t*)lds)[4 * 2048 + blockIdx.x % kPad] = 0;
    const u32 W = gridDim.x * 4u, k = blockIdx.x * 4u + wid;
    constexpr u32 kTot = kNbuf * kTiles;
    const u32 n = k < kTot ? (kTot - k + W - 1u) / W : 0u;
    const u32x4 ri = rsrc(in, 0xFFFFFFF0u);   // (the arena is under 4 GiB)
    uint8_t* my = lds + wid * 2048;
    const u32 l0 = uni(lds_addr(my));
    asm volatile("s_nop 4" ::: "memory");
    if (n > 0) dma(ri, 1024u * k + 16u * lane, l0);
    if (n > 1) dma(ri, 1024u * (k + W) + 16u * lane, l0 + 1024u);
    u32 prev_st = 0;
    for (u32 i = 0; i < n; ++i) {
        vmw(i == 0 ? (n > 1 ? 1u : 0u) : (i + 1u < n ? 1u : 0u) + prev_st);
        const u32 s = i & 1u;
        const u32x4 v = *reinterpret_cast<const u32x4*>(my + s * 1024u + 16u * lane);
        __builtin_amdgcn_s_waitcnt(0xc07f);
        if (i + 2u < n) dma(ri, 1024u * (k + W * (i + 2u)) + 16u * lane, l0 + 1024u * s);
        const u32 g = k + W * i, b = uni(g / kTiles), t = uni(g % kTiles);
        const u32x4 ro = rsrc(out + (uint64_t)b * kOutB, kOutB);
        prev_st = put(ro, t, lane, v);
    }
}

// ---------------------------------------------------------------- copy
template <bool kNt>
__global__ __launch_bounds__(256) void copy_k(u32x4* __restrict__ dst, const u32x4* __restrict__ src, uint64_t n16) {
    const uint64_t stride = (uint64_t)gridDim.x * 1024u;
    for (uint64_t base = (uint64_t)blockIdx.x * 1024u + threadIdx.x; base < n16; base += stride) {
        u32x4 v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint64_t i = base + 256u * q;
            if (i < n16) v[q] = kNt ? __builtin_nontemporal_load(src + i) : src[i];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint64_t i = base + 256u * q;
            if (i < n16) {
                if (kNt) __builtin_nontemporal_store(v[q], dst + i);
                else dst[i] = v[q];
            }
        }
    }
}

template <class F>
static float timeit(F f, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int w = 0; w < 3; ++w) f();
    (void)hipDeviceSynchronize();
    float best = 1e30f;
    for (int round = 0; round < 3; ++round) {
        (void)hipEventRecord(a, 0);
        for (int r = 0; r < reps; ++r) f();
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        best = ms / reps < best ? ms / reps : best;
    }
    return best;
}
static double g_bytes;
static void report(const char* name, float ms) {
    const double tbs = g_bytes / (ms * 1e-3) / 1e12;
    printf("%-52s %8.1f us  %.3f TB/s  frac %.3f\n", name, ms * 1e3, tbs, tbs / 8.0);
    fflush(stdout);
}
template <class K>
static int resident(K kern, int threads) {
    int per = 0, cus = 0, dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)kern, threads, 0);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    return per * cus;
}

int main() {
    uint8_t *in, *out;
    const size_t inb = (size_t)kNbuf * kInB, outb = (size_t)kNbuf * kOutB;
    if (hipMalloc(&in, inb) != hipSuccess || hipMalloc(&out, outb) != hipSuccess) return 1;
    (void)hipMemset(in, 1, inb);
    (void)hipMemset(out, 0, outb);
    (void)hipDeviceSynchronize();
    g_bytes = (double)inb + (double)outb;
    printf("batch: %u buffers, %u KiB in, %u KiB out each; %.3f GB moved per launch\n", kNbuf, kInB / 1024, kOutB / 1024, g_bytes / 1e9);
    const int reps = 10;
    // decode_kernel<96>: ~22.6 KB per 4-wave workgroup (7 per CU); pads below bring each variant there
    report("A  one wave per buffer (7 WG/CU)", timeit([&] { hipLaunchKernelGGL(pat_a<14500>, dim3(kNbuf / 4), dim3(256), 0, 0, in, out); }, reps));
    report("A  one wave per buffer (16 WG/CU cap)", timeit([&] { hipLaunchKernelGGL(pat_a<0>, dim3(kNbuf / 4), dim3(256), 0, 0, in, out); }, reps));
    report("B  4 waves per buffer, interleaved (7 WG/CU)", timeit([&] { hipLaunchKernelGGL(pat_b<14500>, dim3(kNbuf), dim3(256), 0, 0, in, out); }, reps));
    report("B  4 waves per buffer, interleaved (16 WG/CU cap)", timeit([&] { hipLaunchKernelGGL(pat_b<0>, dim3(kNbuf), dim3(256), 0, 0, in, out); }, reps));
    report("C  16-wave rounds per buffer (2 WG/CU)", timeit([&] { hipLaunchKernelGGL((pat_c<16, 40000>), dim3(kNbuf), dim3(1024), 0, 0, in, out); }, reps));
    report("C  16-wave rounds per buffer (no pad)", timeit([&] { hipLaunchKernelGGL((pat_c<16, 0>), dim3(kNbuf), dim3(1024), 0, 0, in, out); }, reps));
    report("C  8-wave rounds per buffer (4 WG/CU)", timeit([&] { hipLaunchKernelGGL((pat_c<8, 24000>), dim3(kNbuf), dim3(512), 0, 0, in, out); }, reps));
    {
        const int g7 = resident(pat_d<14500>, 256), g16 = resident(pat_d<0>, 256), g4 = resident(pat_d<30000>, 256);
        char nm[96];
        snprintf(nm, sizeof nm, "D  arena order, resident grid %d WG (7 WG/CU)", g7);
        report(nm, timeit([&] { hipLaunchKernelGGL(pat_d<14500>, dim3(g7), dim3(256), 0, 0, in, out); }, reps));
        snprintf(nm, sizeof nm, "D  arena order, resident grid %d WG (cap)", g16);
        report(nm, timeit([&] { hipLaunchKernelGGL(pat_d<0>, dim3(g16), dim3(256), 0, 0, in, out); }, reps));
        snprintf(nm, sizeof nm, "D  arena order, resident grid %d WG (4 WG/CU)", g4);
        report(nm, timeit([&] { hipLaunchKernelGGL(pat_d<30000>, dim3(g4), dim3(256), 0, 0, in, out); }, reps));
    }
    {
        // the copy of the same byte count (in + out) / 2 each way
        const uint64_t n16 = (uint64_t)(g_bytes / 2) / 16u;
        uint8_t* big = nullptr;
        if (hipMalloc(&big, 2 * n16 * 16u) == hipSuccess) {
            (void)hipMemset(big, 2, 2 * n16 * 16u);
            const uint64_t want = (n16 + 1023u) / 1024u;
            const u32 grid = (u32)(want < 2048u ? want : 2048u);
            report("copy grid-strided (plain)", timeit([&] { hipLaunchKernelGGL(copy_k<false>, dim3(grid), dim3(256), 0, 0, (u32x4*)(big + n16 * 16u), (const u32x4*)big, n16); }, reps));
            report("copy grid-strided (nt)", timeit([&] { hipLaunchKernelGGL(copy_k<true>, dim3(grid), dim3(256), 0, 0, (u32x4*)(big + n16 * 16u), (const u32x4*)big, n16); }, reps));
            (void)hipFree(big);
        }
    }
    const hipError_t e = hipDeviceSynchronize();
    printf("status: %s\n", hipGetErrorString(e));
    return e == hipSuccess ? 0 : 2;
}
