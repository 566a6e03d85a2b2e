// Small-call latency probe (round 4, host path): one 4 KiB request served (a) by a kernel launch per
// call whose completion flag the host polls (tools/probes/sync_probe.hip mode 1, the drop-in's
// current form) and (b) by a resident one-wave service kernel that polls a mailbox in mapped host
// memory, runs the request and acknowledges it behind a system-scope release -- no launch per call.
// The service kernel ends by itself after `idle` microseconds without a request (and at most `life`
// microseconds after its launch), writing its last served sequence number; the host relaunches it
// when a request finds it gone.  Both modes: 3000 calls of 4 KiB mapped in, 4 KiB mapped out, every
// output word checked; median / mean / p90 microseconds per call, and how many launches the service
// needed.   build: hipcc --offload-arch=gfx950 -O3 tools/probes/mailbox_probe.hip -o build/mailbox_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <chrono>
#include <vector>

constexpr uint32_t kGone = 0xFFFFFFFFu;

__device__ inline uint32_t ld_acq(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ inline void st_rel(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ inline void serve(const uint4* in, uint4* out, uint32_t token) {
    for (uint32_t i = threadIdx.x; i < 256; i += 64) {
        uint4 v = in[i];
        v.x ^= token;
        out[i] = v;
    }
}

__global__ void call_kernel(const uint4* __restrict__ in, uint4* __restrict__ out, uint32_t* ack, uint32_t seq) {
    serve(in, out, seq);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    if (threadIdx.x == 0) __hip_atomic_store(ack, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// box[0] = request sequence (host), box[1] = acknowledged sequence (device), box[2] = the service's
// exit mark (device: last served sequence; kGone while it runs, set by the host before a launch)
__global__ void service_kernel(const uint4* __restrict__ in, uint4* __restrict__ out, uint32_t* box, uint32_t done,
                               uint64_t idle_ticks, uint64_t life_ticks) {
    const uint64_t t0 = wall_clock64();
    uint64_t last = t0;
    for (uint32_t polls = 0;; ++polls) {   // (polls: a second bound, should the clock not advance)
        const uint32_t s = __builtin_amdgcn_readfirstlane(ld_acq(box + 0));
        const uint64_t now = wall_clock64();
        if (s != done) {
            serve(in, out, s);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            if (threadIdx.x == 0) __hip_atomic_store(box + 1, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            done = s;
            last = now;
        } else if (now - last > idle_ticks || now - t0 > life_ticks || polls > (1u << 26)) {
            if (threadIdx.x == 0) st_rel(box + 2, done);
            return;
        } else {
            __builtin_amdgcn_s_sleep(2);
        }
    }
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void report(const char* name, std::vector<double>& t, uint32_t bad, uint32_t launches) {
    std::sort(t.begin(), t.end());
    double sum = 0;
    for (double x : t) sum += x;
    printf("{\"mode\": \"%s\", \"median_us\": %.2f, \"mean_us\": %.2f, \"p90_us\": %.2f, \"max_us\": %.1f, \"bad_words\": %u, "
           "\"launches\": %u}\n", name, t[t.size() / 2], sum / t.size(), t[t.size() * 9 / 10], t.back(), bad, launches);
    fflush(stdout);
}

int main() {
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
    uint4 *h_in, *h_out, *d_in, *d_out;
    uint32_t *h_box, *d_box;
    if (hipHostMalloc((void**)&h_in, 4096, hipHostMallocMapped) != hipSuccess ||
        hipHostMalloc((void**)&h_out, 4096, hipHostMallocMapped) != hipSuccess ||
        hipHostMalloc((void**)&h_box, 256, hipHostMallocMapped) != hipSuccess)
        return 1;
    (void)hipHostGetDevicePointer((void**)&d_in, h_in, 0);
    (void)hipHostGetDevicePointer((void**)&d_out, h_out, 0);
    (void)hipHostGetDevicePointer((void**)&d_box, h_box, 0);
    volatile uint32_t* box = h_box;
    const int N = 3000, W = 300;
    // (a) one launch per call, completion polled
    {
        std::vector<double> t;
        uint32_t bad = 0;
        for (int it = 0; it < N; ++it) {
            const uint32_t seq = 0x1000u + (uint32_t)it;
            for (int i = 0; i < 256; ++i) h_in[i] = make_uint4(i, it, 7, 9);
            box[1] = 0;
            const double t0 = now_us();
            hipLaunchKernelGGL(call_kernel, dim3(1), dim3(64), 0, s, d_in, d_out, d_box + 1, seq);
            while (__atomic_load_n(&box[1], __ATOMIC_ACQUIRE) != seq) {}
            const double t1 = now_us();
            for (int i = 0; i < 256; ++i)
                if (h_out[i].x != ((uint32_t)i ^ seq) || h_out[i].y != (uint32_t)it) ++bad;
            if (it >= W) t.push_back(t1 - t0);
            if ((it & 31) == 31) (void)hipStreamSynchronize(s);
        }
        (void)hipStreamSynchronize(s);
        report("launch per call, polled", t, bad, N);
    }
    // (b) resident service; (c) the same with a short lifetime (relaunches under load)
    for (int mode = 0; mode < 2; ++mode) {
        const uint64_t idle = 100 * 2000, life = mode == 0 ? 100ull * 1000000 : 100ull * 200;   // 100 MHz ticks
        std::vector<double> t;
        uint32_t bad = 0, launches = 0, done = 0;
        box[0] = 0; box[1] = 0; box[2] = 0;   // (exit mark "0": no service running)
        bool running = false;
        for (int it = 0; it < N; ++it) {
            const uint32_t seq = (uint32_t)it + 1u;
            for (int i = 0; i < 256; ++i) h_in[i] = make_uint4(i, it, 7, 9);
            const double t0 = now_us();
            __atomic_store_n(&box[0], seq, __ATOMIC_RELEASE);
            for (;;) {
                if (__atomic_load_n(&box[1], __ATOMIC_ACQUIRE) == seq) break;
                const uint32_t ex = __atomic_load_n(&box[2], __ATOMIC_ACQUIRE);
                if (!running || (ex != kGone && ex != seq)) {   // no service, or it left before this request
                    (void)hipStreamSynchronize(s);                 // (its exit is complete)
                    if (__atomic_load_n(&box[1], __ATOMIC_ACQUIRE) == seq) break;
                    box[2] = kGone;
                    hipLaunchKernelGGL(service_kernel, dim3(1), dim3(64), 0, s, d_in, d_out, d_box, done, idle, life);
                    running = true;
                    ++launches;
                }
            }
            done = seq;
            const double t1 = now_us();
            for (int i = 0; i < 256; ++i)
                if (h_out[i].x != ((uint32_t)i ^ seq) || h_out[i].y != (uint32_t)it) ++bad;
            if (it >= W) t.push_back(t1 - t0);
        }
        // stop: wait for the service's idle exit
        const double tw = now_us();
        (void)hipStreamSynchronize(s);
        printf("{\"exit_wait_us\": %.1f}\n", now_us() - tw);
        report(mode == 0 ? "resident service" : "resident service, 200 us lifetime", t, bad, launches);
    }
    return 0;
}
