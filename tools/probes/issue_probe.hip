// Store-issue probe: does a wave's buffer_store wait behind its own younger load?
// Each wave loops: [load 1 KiB of the next tile] -> ~N dependent VALU -> s_memtime -> store 1 KiB
// -> s_memtime, like one codec tile step, with 16 waves per CU (dynamic LDS sized like decode).
// Reports the mean cycles the store instruction took to issue, and the kernel's bandwidth.
//   mode 0: LDS-DMA load (buffer_load_dwordx4 ... lds)   mode 1: buffer_load_dwordx4 into VGPRs
//   mode 2: no load                                        mode 3: LDS-DMA load, issued AFTER the store
// build: hipcc --offload-arch=gfx950 -O3 tools/probes/issue_probe.hip -o build/issue_probe
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
__device__ __forceinline__ uint64_t stamp() {
    uint64_t t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

template <int kMode, int kWork>
__global__ __launch_bounds__(256) void probe(uint8_t* out, const uint8_t* in, u32 region,
                                             unsigned long long* acc) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const u32 lane = threadIdx.x & 63, wid = (u32)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint64_t w = (uint64_t)blockIdx.x * 4 + wid;
    const u32x4 ro = rsrc(out + w * region, region);
    const u32x4 ri = rsrc(in + w * region, region);
    const u32 l0 = (u32)__builtin_amdgcn_readfirstlane(
        (int)(u32)(uintptr_t)(const __attribute__((address_space(3))) void*)(lds + wid * 9600));
    u32x4 v = {lane, (u32)w, 0x55u, 0xAAu};
    u32x4 r = {0, 0, 0, 0};
    uint64_t st = 0;
    asm volatile("s_nop 4" ::: "memory");
    for (u32 off = 0; off < region; off += 1024) {
        const u32 vo = off + 16 * lane;
        if (kMode == 0) {
            u32 keep;
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
                         : "=&s"(keep) : "v"(vo), "s"(l0), "s"(ri) : "memory");
        } else if (kMode == 1) {
            asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(r) : "v"(vo), "s"(ri) : "memory");
        }
        u32 x = v.z;
#pragma unroll
        for (int k = 0; k < kWork; ++k) x = x * 3u + (u32)k;   // dependent VALU chain
        v.z = x;
        const uint64_t a = stamp();
        asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen" ::"v"(v), "v"(vo), "s"(ro) : "memory");
        const uint64_t b = stamp();
        st += b - a;
        if (kMode == 3) {
            u32 keep;
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
                         : "=&s"(keep) : "v"(vo), "s"(l0), "s"(ri) : "memory");
        }
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");   // keep a few ops in flight, like the codec
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (kMode == 1) v.w += r.x;
    if (lane == 0) atomicAdd(acc, (unsigned long long)st);
    if (lane == 0 && v.w == 0xFFFFFFFFu) out[0] = 1;
}

template <int kMode, int kWork>
void run(uint8_t* out, const uint8_t* in, u32 waves, u32 region, unsigned long long* acc) {
    (void)hipMemset(acc, 0, 8);
    hipLaunchKernelGGL((probe<kMode, kWork>), dim3(waves / 4), dim3(256), 4 * 9600, 0, out, in, region, acc);
    (void)hipDeviceSynchronize();
    (void)hipMemset(acc, 0, 8);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL((probe<kMode, kWork>), dim3(waves / 4), dim3(256), 4 * 9600, 0, out, in, region, acc);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h = 0;
    (void)hipMemcpy(&h, acc, 8, hipMemcpyDeviceToHost);
    const double stores = (double)waves * (region / 1024);
    const double bytes = (double)waves * region * (kMode == 2 ? 1 : 2);
    printf("mode %d work %4d: store issue %7.0f cyc | %6.0f GB/s (%s)\n", kMode, kWork, h / stores,
           bytes / ms / 1e6, kMode == 2 ? "w" : "r+w");
}

int main() {
    const u32 region = 64 * 1024, waves = 16384;
    const size_t bytes = (size_t)waves * region;
    uint8_t *out, *in;
    unsigned long long* acc;
    if (hipMalloc(&out, bytes) != hipSuccess || hipMalloc(&in, bytes) != hipSuccess || hipMalloc(&acc, 8) != hipSuccess)
        return 1;
    (void)hipMemset(in, 1, bytes);
    run<0, 64>(out, in, waves, region, acc);
    run<1, 64>(out, in, waves, region, acc);
    run<2, 64>(out, in, waves, region, acc);
    run<3, 64>(out, in, waves, region, acc);
    run<0, 512>(out, in, waves, region, acc);
    run<1, 512>(out, in, waves, region, acc);
    run<2, 512>(out, in, waves, region, acc);
    run<3, 512>(out, in, waves, region, acc);
    return 0;
}
