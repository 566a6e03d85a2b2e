// Hardware-queue probe (round 4, host path): does a long-running kernel on a high-priority stream
// hold up kernels on the process's normal-priority streams?  HIP maps streams onto a few hardware
// queues (GPU_MAX_HW_QUEUES, default 4); streams sharing a queue run in its order.  A spin kernel
// (one wave, ends by itself after `ms` milliseconds of the GPU's wall clock) is launched on a
// stream of the given priority, then a tiny kernel on each of 12 fresh normal-priority streams; the
// host times each tiny kernel's completion.  A completion near `ms` means that stream shares the
// spinner's queue.   build: hipcc --offload-arch=gfx950 -O3 tools/probes/queue_probe.hip -o build/queue_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <chrono>

__global__ void spin_kernel(uint64_t ticks) {
    const uint64_t t0 = wall_clock64();
    for (uint32_t i = 0; i < (1u << 26); ++i) {   // (i: a second bound, should the clock not advance)
        if (wall_clock64() - t0 > ticks) break;
        __builtin_amdgcn_s_sleep(8);
    }
}
__global__ void tiny_kernel(uint32_t* p) {
    if (threadIdx.x == 0) p[blockIdx.x] = 1u;
}

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    int lo = 0, hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
    printf("{\"priority_range\": [%d, %d]}\n", lo, hi);
    uint32_t* d = nullptr;
    if (hipMalloc(&d, 4096) != hipSuccess) return 1;
    // variants: the spinner at the greatest / least / the default priority (the normal streams' own);
    // `dep`: each normal stream launches two tiny kernels back to back (the second waits for the first
    // in its stream), as the drop-in's multi-launch calls do, instead of one
    const int prios[3] = {hi, lo, 0};
    for (int variant = 0; variant < 6; ++variant) {
        const int prio = prios[variant % 3];   // hi = the greatest priority (numerically lowest)
        const bool dep = variant >= 3;
        hipStream_t sp;
        if (hipStreamCreateWithPriority(&sp, hipStreamNonBlocking, prio) != hipSuccess) return 1;
        hipStream_t s[12];
        for (int i = 0; i < 12; ++i)
            if (hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking) != hipSuccess) return 1;
        tiny_kernel<<<1, 64, 0, sp>>>(d);   // warm up both kernels
        (void)hipStreamSynchronize(sp);
        const double spin_ms = 20.0;
        const double t0 = now_ms();
        spin_kernel<<<1, 64, 0, sp>>>((uint64_t)(spin_ms * 100000.0));   // 100 MHz ticks
        double done[12];
        for (int i = 0; i < 12; ++i) {
            tiny_kernel<<<1, 64, 0, s[i]>>>(d + 64 * i);
            if (dep) tiny_kernel<<<1, 64, 0, s[i]>>>(d + 64 * i);
        }
        for (int i = 0; i < 12; ++i) {
            (void)hipStreamSynchronize(s[i]);
            done[i] = now_ms() - t0;
        }
        (void)hipStreamSynchronize(sp);
        const double spin_done = now_ms() - t0;
        printf("{\"spinner_priority\": %d, \"dependent_pair\": %s, \"spin_ms\": %.1f, \"spinner_done_ms\": %.2f, \"tiny_done_ms\": [",
               prio, dep ? "true" : "false", spin_ms, spin_done);
        for (int i = 0; i < 12; ++i) printf("%s%.2f", i ? ", " : "", done[i]);
        printf("]}\n");
        fflush(stdout);
        for (int i = 0; i < 12; ++i) (void)hipStreamDestroy(s[i]);
        (void)hipStreamDestroy(sp);
    }
    return 0;
}
