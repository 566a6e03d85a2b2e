// rle_dropin.cpp — the drop-in C ABI of include/rleCompression.h on top of the MI355X kernels.
//
// Replaces src/rleCompression.c:9-62 (samul-1/C-FileStorage-Server-and-Client) for its callers
// src/filesystemApi.c:597 (read), :680 (readNFiles), :767/:774 (write/append = decode, append,
// re-encode) and src/server.c:317 (evicted files), which link against this library unchanged.
//
// Each calling thread (the server's worker pool, src/server.c:520-524) gets its own HIP stream,
// pinned host buffers and device buffers, created lazily on its first call (there is no init
// hook in the server, src/server.c:406-524) and released at thread exit.  A call is one batched
// kernel launch with B = 1 plus the host<->device traffic, sized to the call:
//   small (one wave walks it)  zero-copy on the thread's mapped pinned buffer, one launch, one sync;
//   medium (up to 256 KiB)     zero-copy too: cooperative or segmented kernels on the mapped buffer;
//   large                      the caller's buffer and the result block registered for the call, one
//                              DMA in, segmented kernels, one copy kernel out (else the runtime's
//                              pageable copies or the pinned staging).
// The result is a fresh malloc() block, which is what the callers free() (src/filesystemApi.c:208,
// 687, 775, 811; src/server.c:269, 320).  There is no CPU codec in this library: without a
// usable GPU it reports the problem and aborts.  RLEappend / RLEdecompressN (include/
// rle_fileops.h) are the fused and batched forms of the callers' compositions.
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <sched.h>
#include <errno.h>
#include <link.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <new>
#include <mutex>
#include <vector>

#include "rleCompression.h"
#include "rle_fileops.h"
#include "rle_mi355x.h"
#include "rle_service.h"
#include "rle_build.h"
#include "rle_coop_limits.h"

// Measured-slower host-path variants (call coalescing, pipelined staging) are compiled only into the
// test library (build/librle_mi355x_testhooks.so) and `make variant` builds, never into the product
// librle_mi355x.so (the measurements are in DESIGN.md §6).

namespace {

pthread_once_t g_once = PTHREAD_ONCE_INIT;
pthread_key_t g_key;
int g_ndev = 0;
int g_dev_pin = -1;
std::atomic<unsigned> g_next_dev{0};
std::atomic<int> g_warned_overflow{0};

// Host-path accounting (rle_mi355x_dropin_stats): bytes moved and wall time per phase.
struct Stats {
    std::atomic<uint64_t> calls_compress{0}, calls_decompress{0}, calls_append{0};
    std::atomic<uint64_t> bytes_in{0}, bytes_out{0};        // caller bytes in / returned bytes out
    std::atomic<uint64_t> bytes_h2d{0}, bytes_d2h{0};
    std::atomic<uint64_t> ns_stage_in{0}, ns_device{0}, ns_stage_out{0};
    std::atomic<uint64_t> calls_coalesced{0}, launches_coalesced{0};   // zero-copy calls / their combined launches
    std::atomic<uint64_t> calls_registered{0}, calls_reg_fallback{0};  // registered large calls / staged instead
} g_stats;
inline uint64_t now_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}

// RLE_MI355X_TRACE=<path> (diagnostics of the e2e batteries): one record per drop-in
// call -- the entry point, its sizes, start and duration, the calling thread and the time it spent
// getting its context (pool wait or creation) -- written to <path> at exit.  Off: one branch per call.
struct TraceRec {
    char op;
    uint32_t tid;
    uint64_t a, b, c, t0, dt, ctx_ns;
};
constexpr uint32_t kTraceMax = 1u << 16;
TraceRec* g_trace = nullptr;
std::atomic<uint32_t> g_trace_n{0};
thread_local uint64_t t_ctx_ns = 0;
struct TraceScope {
    char op;
    uint64_t a, b, c, t0;
    TraceScope(char o, uint64_t x, uint64_t y, uint64_t z) : op(o), a(x), b(y), c(z), t0(g_trace ? now_ns() : 0) {
        t_ctx_ns = 0;
    }
    ~TraceScope() {
        if (!g_trace) return;
        const uint32_t i = g_trace_n.fetch_add(1, std::memory_order_relaxed);
        if (i < kTraceMax) g_trace[i] = TraceRec{op, (uint32_t)syscall(SYS_gettid), a, b, c, t0, now_ns() - t0, t_ctx_ns};
    }
};

[[noreturn]] void die(const char* what, hipError_t e) {
    fprintf(stderr, "librle_mi355x: %s failed: %s\n", what, hipGetErrorString(e));
    abort();
}
inline void check(hipError_t e, const char* what) {
    if (e != hipSuccess) die(what, e);
}
// Buffers past RLE_MAX_BUFFER_BYTES (2 GiB) are not handled by the kernels: the call fails with
// errno = EFBIG (reported once on stderr) instead of returning a wrong result.
std::atomic<int> g_warned_big{0};
bool too_big(const char* who, size_t n) {
    if (n <= RLE_MAX_BUFFER_BYTES) return false;
    if (!g_warned_big.exchange(1))
        fprintf(stderr, "librle_mi355x: %s: %zu bytes exceeds the per-buffer limit of %u\n", who, n,
                (unsigned)RLE_MAX_BUFFER_BYTES);
    errno = EFBIG;
    return true;
}

// Small-call threshold: up to this many input bytes the worst-case output is copied back in the
// same round trip as its size (one stream sync instead of two).
constexpr size_t kOneTripBytes = 128u << 10;
// From these sizes one call is cut into segments processed by separate waves
// (rle_*_batch_device_seg) instead of one wave walking the whole buffer.
constexpr size_t kSegEncodeBytes = 48u << 10;
constexpr size_t kSegDecodeBytes = 32u << 10;

// Host<->device transfers of large calls, selected by RLE_MI355X_STAGING:
//   direct (default) the HIP runtime copies from / to the caller's pageable memory itself;
//   pinned one memcpy into / out of this thread's pinned staging, one DMA;
//   pipe   the pinned staging in chunks, the memcpy of one chunk overlapping the DMA of the next.
// Calls below kPipeMinBytes always take "pinned" (one DMA each way).  Measured on MI355X
// (profiles/r1d_staging.md): at 4 MiB, direct takes 231 / 255 us per compress / decompress call,
// pinned 424 / 470, pipe 489 / 567; from 64 KiB to 1 MiB the three are within a few percent.
enum class Staging { Pinned, Pipe, Direct };
Staging g_staging = Staging::Direct;
constexpr size_t kPipeMinBytes = 256u << 10;
constexpr int kPipeEvents = 16;

// Small calls run zero-copy by default: the kernel reads the caller's bytes from, and writes its
// result into, this thread's mapped pinned buffer over PCIe, with no copy commands at all (4 KiB:
// 19 / 20 us per compress / decompress call against 21 / 23 with one H2D + one D2H;
// profiles/r1e_small.md).  RLE_MI355X_SMALL=copy selects the copying form.
bool g_zerocopy = true;
#if RLE_VARIANTS
bool g_coalesce = false;   // concurrent zero-copy calls join one launch (submit); RLE_MI355X_COALESCE=1: on
#endif
size_t g_presize = 1u << 20;   // staging allocated with each thread context (presize); RLE_MI355X_PRESIZE
// Zero-copy calls learn of their completion from the status word the kernel stores last, behind a
// system-scope release of its output (RLE_LAUNCH_STATUS_FLAG), by polling it in the mapped buffer
// instead of hipStreamSynchronize (profiles/r4a_sync_probe.txt: 11.7 against 16.2 us per 4 KiB
// launch).  RLE_MI355X_POLL=0: synchronize instead.
bool g_poll = true;
// How long a completion poll spins (pause) before it yields the core between reads:
// RLE_MI355X_SPIN_NS (default 50 us, about the longest small call).
uint64_t g_spin_ns = 50000;
// Small calls through the resident service (rle_service.h) instead of a launch each:
// RLE_MI355X_SERVICE=1, in the RLE_VARIANTS test library only (measured slower, round 5).
bool g_service = false;
// Zero-copy calls from this many bytes (encode: U, decode: C) run the segmented kernels on the mapped
// buffer instead of one wave walking it, and the zero-copy form then takes calls up to 256 KiB in
// (RLE_MI355X_ZC_SEG=<bytes>; 0 = never).  profiles/r4f_callrate_zcseg.txt, µs per call on 1 / 8
// threads: 40 KB 42.2 / 91.7 against 66.1 / 151.3 for one wave over the mapped buffer; 24 KiB
// 41.2 / 91.1 against 34.8 / 64.2 (the five launches cost more than a short walk).
size_t g_zc_seg = 32u << 10;
// ... except the calls one cooperative workgroup takes (rle_coop_limits.h: encode up to 64 KiB,
// decode up to 80 tiles decoding to 64 KiB; rounds of 16 waves, one launch, polled like the smaller
// calls).  RLE_MI355X_ZC_COOP=0: the segmented kernels from g_zc_seg as before (round 5 A/B).
bool g_zc_coop = true;
// Input up to 256 KiB, output up to 384 KiB (r5n / r5o, profiles/r5o_zc_size.md: past the cooperative
// kernels' reach the segmented kernels on the mapped buffer beat the two copies of the staged path up
// to 256 KiB, e.g. a 96 KiB compress 43 against 68 us; 80 KiB of input until round 5's r5n)
#ifndef RLE_ZC_IN_KIB
#define RLE_ZC_IN_KIB 256
#endif
constexpr size_t kZcIn = 0, kZcWords = (size_t)RLE_ZC_IN_KIB << 10, kZcOut = kZcWords + (4u << 10),
                 kZcBytes = kZcOut + (kZcWords * 3 / 2 > (204u << 10) ? kZcWords * 3 / 2 : (204u << 10));
static_assert(kZcWords >= rle::kCoopDecMaxIn, "zero-copy input region");
constexpr size_t kZcMaxIn = kZcWords, kZcMaxOut = kZcBytes - kZcOut;   // one zero-copy call's bytes

// Registered large calls (profiles/r6j_hostpath_reg.txt, r6_hostpath.md): from
// g_reg_min bytes (RLE_MI355X_REG_MIN; 0 = never; by default the sizes past the zero-copy calls'
// reach) an RLEcompress / RLEdecompress registers the caller's input and the result block with the
// runtime for the duration of the call (hipHostRegister + unregister of 1 MiB of touched heap
// memory: 0.9 + 0.3 µs).  The input travels by one DMA straight from the caller's pages, the kernels
// work in device memory, and a copy kernel stores the result into the registered block over PCIe
// (the write pass storing there itself measured slower: its partial lines, r6k): no CPU copy either
// way, and a compress reads its output length on the device instead of a second round trip.  1 MiB:
// 83-89 µs per call against 111-140 through the runtime's pageable copies.
//
// Only a call that is the only large call in flight registers (LargeCall): registered calls from
// several threads at once measured slower than the pageable copies (r6p: 8 threads, 1 MiB round
// trips, 6.9 against 13.4 GB/s in round 5), and a registration must never meet a pageable copy of
// the same pages by the runtime (another thread's call on the same stored file), whose pinning in
// place races the unregistration (r6q: a crash).  So the decision is taken under g_reg_mu together
// with the count of large calls in flight (no registration starts while another large call is in
// flight), and a transfer whose caller pages meet a live registration's pages goes through the
// pinned staging, never handing the runtime that pointer (live_pages).
size_t g_reg_min = kZcMaxIn + 1;   // (past the zero-copy calls: r6m / r6o)
std::mutex g_reg_mu;
std::atomic<int> g_large_calls{0};       // large calls in flight (changed under g_reg_mu)
// ... and when two last overlapped: a call registers only when none has overlapped it for
// kRegQuietNs (RLE_MI355X_REG_QUIET_US).  Under a steady multi-threaded load the registering calls
// that happen to run alone still cost the others (their registration and unregistration), 4
// threads of 1 MiB round trips 7.5-7.8 against 8.7-9.4 GB/s (r6t).
std::atomic<uint64_t> g_last_overlap_ns{0};
uint64_t g_reg_quiet_ns = 2000000;
// Whether a call starting now would register (read without the lock: a hint, so that a call that
// will not register does not allocate its worst-case result block first).
bool reg_likely() {
    return g_large_calls.load(std::memory_order_relaxed) == 0 &&
           now_ns() - g_last_overlap_ns.load(std::memory_order_relaxed) > g_reg_quiet_ns;
}
int g_live_regs = 0;                     // registrations alive (under g_reg_mu)
uintptr_t g_live_lo[2], g_live_hi[2];    // the registered call's page spans (under g_reg_mu)
inline uintptr_t page_lo(const void* p) { return (uintptr_t)p & ~(uintptr_t)4095; }
inline uintptr_t page_hi(const void* p, size_t n) { return ((uintptr_t)p + n + 4095) & ~(uintptr_t)4095; }
// Whether host bytes [p, p + n) share a page with a live registration.
bool live_pages(const void* p, size_t n) {
    std::lock_guard<std::mutex> g(g_reg_mu);
    const uintptr_t lo = page_lo(p), hi = page_hi(p, n);
    for (int i = 0; i < g_live_regs; ++i)
        if (lo < g_live_hi[i] && g_live_lo[i] < hi) return true;
    return false;
}

// hipHostRegister of [p, p + n) and its device address (nullptr: not registered).  Under g_reg_mu.
uint8_t* reg_one(const void* p, size_t n, bool read_only) {
    void* q = const_cast<void*>(p);
    hipError_t e = hipHostRegister(q, n, hipHostRegisterMapped | (read_only ? hipHostRegisterReadOnly : 0u));
    if (e != hipSuccess && read_only) {   // (read-only pages that the flag is not supported for)
        (void)hipGetLastError();
        e = hipHostRegister(q, n, hipHostRegisterMapped);
    }
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    void* d = nullptr;
    // (the result block's device address must be 16-byte aligned for the copy kernel; the input
    // travels by DMA from its host address)
    if (hipHostGetDevicePointer(&d, q, 0) != hipSuccess || !d || (!read_only && ((uintptr_t)d & 15u))) {
        (void)hipGetLastError();
        (void)hipHostUnregister(q);
        return nullptr;
    }
    g_live_lo[g_live_regs] = page_lo(p);
    g_live_hi[g_live_regs] = page_hi(p, n);
    ++g_live_regs;
    return static_cast<uint8_t*>(d);
}
void unreg_all(const void* in, const void* out) {   // (the registered call's two, in that order)
    (void)hipHostUnregister(const_cast<void*>(out));
    (void)hipHostUnregister(const_cast<void*>(in));
    (void)hipGetLastError();
    g_live_regs = 0;
}

// One drop-in call that moves caller bytes past the zero-copy reach, from before its first
// transfer to after its last.  Constructed with an input and a result block, it registers both
// when it is the only large call in flight (registered(); d_in / d_out their device addresses).
// Leaving, it drains the call's stream before unregistering (a call left by an exception).
class LargeCall {
public:
    explicit LargeCall(hipStream_t s, const void* in = nullptr, size_t n_in = 0, const void* out = nullptr,
                       size_t n_out = 0)
        : s_(s) {
        std::lock_guard<std::mutex> g(g_reg_mu);
        const uint64_t t = now_ns();
        const int n = ++g_large_calls;
        if (n > 1) g_last_overlap_ns = t;
        if (in && n == 1 && t - g_last_overlap_ns > g_reg_quiet_ns && (d_in = reg_one(in, n_in, true))) {
            // (the input and the result block may share a page when malloc put them side by side:
            // a read-only and a read-write registration of one page measured correct,
            // tools/probes/reg_shared_page_probe.hip, r6ao)
            if ((d_out = reg_one(out, n_out, false))) {
                in_ = in;
                out_ = out;
            } else {
                (void)hipHostUnregister(const_cast<void*>(in));
                (void)hipGetLastError();
                g_live_regs = 0;
                d_in = nullptr;
            }
        }
    }
    ~LargeCall() {
        if (registered()) (void)hipStreamSynchronize(s_);
        std::lock_guard<std::mutex> g(g_reg_mu);
        if (registered()) unreg_all(in_, out_);
        --g_large_calls;
    }
    LargeCall(const LargeCall&) = delete;
    LargeCall& operator=(const LargeCall&) = delete;
    bool registered() const { return d_out != nullptr; }
    uint8_t* d_in = nullptr;
    uint8_t* d_out = nullptr;

private:
    hipStream_t s_;
    const void* in_ = nullptr;
    const void* out_ = nullptr;
};

// Pinned staging of RLEdecompressN is bounded: a batch is processed in chunks of at most this many
// staged input (and output) bytes, and a file larger than that is copied straight from / to the
// caller's memory, so a readN of the whole store does not pin the store's size per worker thread.
// RLE_MI355X_STAGE_CAP=<bytes> overrides it (tests use small caps to cover the chunking).
size_t g_stage_cap = 32u << 20;

// Test builds only (RLE_TEST_HOOKS=1: build/librle_mi355x_testhooks.so, never the product library):
// RLE_MI355X_FAIL_ALLOC_ABOVE=<bytes> makes staging / device allocations larger than that fail as
// if memory were exhausted, so the allocation-failure paths can be exercised.
#if RLE_TEST_HOOKS
size_t g_fail_above = SIZE_MAX;
inline bool injected_failure(size_t n) { return n > g_fail_above; }
// RLE_MI355X_FAKE_DEVICES=<n> (CPU lifecycle tests, tests/test_lifecycle.py): the library believes n
// devices exist and builds thread contexts that hold no HIP object (no HIP call is made for them),
// so the start-up thread, the pool, the pthread-key destructors, fork and exit ordering all run on a
// machine without a GPU, under ASan and TSan.  RLE_MI355X_FAKE_DELAY_US: each context takes that long.
int g_fake_devs = 0;
unsigned g_fake_delay_us = 0;
#else
constexpr bool injected_failure(size_t) { return false; }
constexpr int g_fake_devs = 0;
constexpr unsigned g_fake_delay_us = 0;
#endif

struct Ctx {
    int dev = 0;
    uint8_t* h_zc = nullptr;                         // mapped pinned buffer of the zero-copy calls
    uint8_t* d_zc = nullptr;                         // its device address
    hipEvent_t ev[kPipeEvents] = {};                 // chunk completion events of the pipelined D2H
    hipStream_t s = nullptr;
    uint8_t* h_in = nullptr;  size_t h_in_cap = 0;    // pinned staging: caller bytes -> device
    uint8_t* h_out = nullptr; size_t h_out_cap = 0;   // pinned staging: device -> caller block
    uint8_t* d_in = nullptr;  size_t d_in_cap = 0;
    uint8_t* d_out = nullptr; size_t d_out_cap = 0;
    uint64_t* d_meta = nullptr;                      // kMetaSlots u64: per-launch [in_off, in_len, out_off, ...]
    uint64_t* h_meta = nullptr;                      // pinned mirror
    uint8_t* d_ws = nullptr;  size_t d_ws_cap = 0;    // segmented-path workspace
    uint8_t* d_mid = nullptr; size_t d_mid_cap = 0;   // RLEappend: decoded old content ‖ new bytes
    uint8_t* h_bm = nullptr;  size_t h_bm_cap = 0;    // RLEdecompressN: per-file offsets/lengths/status
    uint8_t* d_bm = nullptr;  size_t d_bm_cap = 0;
    uint8_t* h_cw = nullptr;                         // mapped launch words of combined launches (submit)
    uint8_t* d_cw = nullptr;
    uint32_t polled = 0;                             // polled launches since the last stream synchronize
    int svc = -2;                                    // resident service (rle_service.h): 1 on, -1 off, -2 not yet asked
    rle::SvcMail* svc_h = nullptr;                   // its mailbox (in the mapped zero-copy buffer) ...
    rle::SvcMail* svc_d = nullptr;                   // ... and the mailbox's device address
    hipStream_t svc_s = nullptr;                     // the service's stream
    uint32_t svc_seq = 0;                            // latest request
    uint32_t svc_gen = 0;                            // latest launch (0: none)
    bool full = false;                               // presized and warmed for large calls (preinit)
};
// h_meta / d_meta regions, one per launch that can be in flight on the stream at once:
//   decode [in_off, in_len, out_off, out_len, out_cap, status], encode [in_off, in_len, out_off,
//   out_len, -, status], append (rle_append_prepare_device's 4 u64)
constexpr size_t kMetaDec = 0, kMetaEnc = 8, kMetaApp = 16, kMetaSlots = 24;

// A worker thread's context is released by its pthread-key destructor, which can still be running
// when the process exits (a thread joined by its creator has not necessarily finished its TLS
// destructors).  Process exit tears the HIP runtime down, so from the first atexit handler on no
// context touches HIP any more (the OS reclaims the memory); the lock orders the two.
pthread_mutex_t g_exit_lock = PTHREAD_MUTEX_INITIALIZER;
bool g_exiting = false;
void preinit_join();   // below
void svc_stop();   // below
void svc_end(Ctx* c);
void svc_unregister(Ctx* c);
void on_exit_handler() {
    preinit_join();   // (when called from the start-up thread's own exit: never; it makes no exit call)
    svc_stop();
    pthread_mutex_lock(&g_exit_lock);
    g_exiting = true;
    pthread_mutex_unlock(&g_exit_lock);
}

void free_ctx(void* p) {
    Ctx* c = static_cast<Ctx*>(p);
    if (!c) return;
    pthread_mutex_lock(&g_exit_lock);
    if (g_exiting) {
        pthread_mutex_unlock(&g_exit_lock);
        return;
    }
    if (g_fake_devs) {   // (test build: a context without HIP objects)
        delete c;
        pthread_mutex_unlock(&g_exit_lock);
        return;
    }
    (void)hipSetDevice(c->dev);
    svc_end(c);
    svc_unregister(c);
    if (c->s) (void)hipStreamSynchronize(c->s);
    (void)hipHostFree(c->h_in);
    (void)hipHostFree(c->h_out);
    (void)hipHostFree(c->h_meta);
    (void)hipHostFree(c->h_bm);
    (void)hipHostFree(c->h_zc);
    (void)hipHostFree(c->h_cw);
    (void)hipFree(c->d_in);
    (void)hipFree(c->d_out);
    (void)hipFree(c->d_meta);
    (void)hipFree(c->d_ws);
    (void)hipFree(c->d_mid);
    (void)hipFree(c->d_bm);
    for (hipEvent_t e : c->ev)
        if (e) (void)hipEventDestroy(e);
    if (c->s) {
        (void)rle_decode_release_stream(c->s);   // (the issue-order array of large RLEdecompressN batches)
        (void)hipStreamDestroy(c->s);
    }
    delete c;
    pthread_mutex_unlock(&g_exit_lock);
}

void init_once() {
#if RLE_TEST_HOOKS
    if (const char* e = getenv("RLE_MI355X_FAKE_DEVICES")) g_fake_devs = atoi(e) > 0 ? atoi(e) : 0;
    if (const char* e = getenv("RLE_MI355X_FAKE_DELAY_US")) g_fake_delay_us = (unsigned)atoi(e);
#endif
    if (g_fake_devs) g_ndev = g_fake_devs;
    else if (hipGetDeviceCount(&g_ndev) != hipSuccess) g_ndev = 0;
    if (const char* e = getenv("RLE_MI355X_DEVICE")) g_dev_pin = atoi(e);
    if (const char* e = getenv("RLE_MI355X_SMALL")) g_zerocopy = strcmp(e, "copy") != 0;
    if (const char* e = getenv("RLE_MI355X_POLL")) g_poll = strcmp(e, "0") != 0;
    if (const char* e = getenv("RLE_MI355X_SPIN_NS")) g_spin_ns = strtoull(e, nullptr, 10);
    if (const char* e = getenv("RLE_MI355X_SERVICE")) g_service = strcmp(e, "0") != 0;
    if (const char* e = getenv("RLE_MI355X_ZC_SEG")) g_zc_seg = (size_t)strtoull(e, nullptr, 10);
    if (const char* e = getenv("RLE_MI355X_ZC_COOP")) g_zc_coop = strcmp(e, "0") != 0;
    if (const char* e = getenv("RLE_MI355X_COOP")) g_zc_coop = g_zc_coop && strcmp(e, "0") != 0;   // (no workgroups to take them)
#if RLE_VARIANTS
    if (const char* e = getenv("RLE_MI355X_COALESCE")) g_coalesce = strcmp(e, "0") != 0;
#endif
    if (const char* e = getenv("RLE_MI355X_PRESIZE")) g_presize = (size_t)strtoull(e, nullptr, 10);
    if (const char* e = getenv("RLE_MI355X_STAGING")) {
        if (!strcmp(e, "pinned")) g_staging = Staging::Pinned;
        else if (RLE_VARIANTS && !strcmp(e, "pipe")) g_staging = Staging::Pipe;
    }
#if RLE_TEST_HOOKS
    if (const char* e = getenv("RLE_MI355X_FAIL_ALLOC_ABOVE")) g_fail_above = (size_t)strtoull(e, nullptr, 10);
#endif
    if (const char* e = getenv("RLE_MI355X_REG_MIN")) g_reg_min = (size_t)strtoull(e, nullptr, 10);
    if (const char* e = getenv("RLE_MI355X_REG_QUIET_US")) g_reg_quiet_ns = 1000ull * strtoull(e, nullptr, 10);
    if (const char* e = getenv("RLE_MI355X_STAGE_CAP")) {
        const long long v = atoll(e);
        if (v >= 16) g_stage_cap = (size_t)v;
    }
    pthread_key_create(&g_key, free_ctx);
    atexit(on_exit_handler);   // registered after the HIP runtime's own exit hooks: runs before them
}

inline size_t round16(size_t x) { return (x + 15u) & ~(size_t)15u; }

void presize(Ctx* c);   // below
void warm(Ctx* c);      // below
void warm_small(Ctx* c);   // below

// A context on device dev: its stream, launch words and (sized) staging.  Throws std::bad_alloc.
Ctx* new_ctx(int dev, bool sized = true) {
    Ctx* c = new Ctx();
    c->dev = dev;
    if (g_fake_devs) {   // (test build: no HIP objects)
        if (g_fake_delay_us) usleep(g_fake_delay_us);
        c->full = sized;
        return c;
    }
    check(hipSetDevice(c->dev), "hipSetDevice");
    check(hipStreamCreateWithFlags(&c->s, hipStreamNonBlocking), "hipStreamCreate");
    if (hipMalloc(&c->d_meta, kMetaSlots * sizeof(uint64_t)) != hipSuccess ||
        hipHostMalloc(&c->h_meta, kMetaSlots * sizeof(uint64_t), hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipFree(c->d_meta);
        (void)hipStreamDestroy(c->s);
        delete c;
        throw std::bad_alloc();
    }
    if (sized) presize(c);
    c->full = sized;
    return c;
}

// ---------------------------------------------------------------- start-up off the call path (r4)
// The server has no init hook (src/server.c:406-524), so until round 3 the first codec call of the
// process paid the HIP runtime's start-up, and every worker thread's first call paid its context
// (stream, pinned and device buffers: hipHostMalloc costs milliseconds) and the first use of the copy
// engines (e2e battery 1: 89-167 ms against the reference's 5-7 ms; ns_stage_in 7.75 ms for 883 KB).
// Now the library's constructor starts one background thread when it is loaded, before main() runs
// in a server that links it (round 5: only a main program that names the library among its DT_NEEDED
// entries, or any process with RLE_MI355X_PREINIT > 0; a process that dlopen()s it, such as Python,
// does not start it unless asked): the thread initialises the runtime and builds RLE_MI355X_PREINIT
// contexts (default 8; 0 = off, the round-3 behaviour) in two phases: first one sized and warmed
// with one call of every transfer form (pinned, pageable) and kernel form, and the others only
// ready for small calls (stream, launch words, zero-copy buffer, one small call each way), each put
// in the pool as soon as it is ready; then those still in the pool sized and warmed too (r4e trace: with one phase, 8 worker threads writing at once on a fresh server
// waited 32, 17, 10, 10, 4, 4 and 4 ms in turn for their contexts, serialised by the store lock).
// A worker's first call takes a context from the pool (waiting for the thread if it is still
// building them), and makes its own only when the pool is empty.  Process exit stops the thread between two steps and
// waits for it (preinit_exit, registered before the thread starts), so it never runs into the
// runtime's teardown.
// Everything the start-up thread touches is constant-initialised (POD, pthread static
// initialisers): the constructor that starts it may run before this file's dynamic initialisers
// (a std::vector pool re-initialised under the running thread corrupted the heap, r4a e2e run).
constexpr int kPoolMax = 64;
pthread_mutex_t g_pool_m = PTHREAD_MUTEX_INITIALIZER;
pthread_cond_t g_pool_cv = PTHREAD_COND_INITIALIZER;
Ctx* g_pool[kPoolMax];
int g_pool_n = 0;                    // under g_pool_m
bool g_pre_running = false;          // under g_pool_m
bool g_pre_phase1 = false;           // under g_pool_m: phase 1 (contexts still being made) running
std::atomic<bool> g_pre_stop{false};
pthread_t g_pre_thread;
std::atomic<bool> g_pre_started{false};

void* preinit_main(void*) {
    int want = 8;
    if (const char* e = getenv("RLE_MI355X_PREINIT")) want = atoi(e);
    want = want < kPoolMax ? want : kPoolMax;
    {
        TraceScope ts('I', 0, 0, 0);   // (trace record: the runtime's start-up)
        pthread_once(&g_once, init_once);
    }
    // phase 1: every context ready for small calls (stream, launch words, zero-copy buffer, one
    // small call each way), so that the worker threads' first calls wait as little as possible
    for (int i = 0; i < want && g_ndev > 0 && !g_pre_stop.load(); ++i) {
        const int dev = (g_dev_pin >= 0 && g_dev_pin < g_ndev) ? g_dev_pin : (int)(g_next_dev++ % (unsigned)g_ndev);
        Ctx* c = nullptr;
        try {
            TraceScope ts('P', 1, (uint64_t)i, 0);   // (trace records: each context's phase-1 set-up ...)
            {
                TraceScope tn('N', 1, (uint64_t)i, 0);   // (... of which making the context)
                c = new_ctx(dev, i == 0);
            }
            // the first context sized and warmed for every call form at once: the process-wide
            // first uses (each kernel's first launch, the runtime's copy paths) are then done before
            // a worker's first large call (r4 e2e: with every context light first, the first large
            // calls spent 26.6 ms staging in against 0.07 ms)
            if (g_fake_devs) {
            } else if (i == 0) warm(c);
            else warm_small(c);
        } catch (const std::bad_alloc&) {
            if (c) free_ctx(c);
            break;
        }
        pthread_mutex_lock(&g_pool_m);
        g_pool[g_pool_n++] = c;
        pthread_cond_broadcast(&g_pool_cv);
        pthread_mutex_unlock(&g_pool_m);
    }
    // phase 2: the contexts still in the pool, one at a time, sized and warmed for large calls (a
    // context a worker has taken meanwhile grows its staging on demand instead).  A worker that
    // finds the pool empty now makes its own context rather than wait for this one (r4f trace).
    pthread_mutex_lock(&g_pool_m);
    g_pre_phase1 = false;
    pthread_cond_broadcast(&g_pool_cv);
    pthread_mutex_unlock(&g_pool_m);
    while (!g_pre_stop.load()) {
        Ctx* c = nullptr;
        pthread_mutex_lock(&g_pool_m);
        for (int i = 0; i < g_pool_n; ++i)
            if (!g_pool[i]->full) {
                c = g_pool[i];
                g_pool[i] = g_pool[--g_pool_n];
                break;
            }
        pthread_mutex_unlock(&g_pool_m);
        if (!c) break;
        try {
            TraceScope ts('P', 2, 0, 0);   // (trace record: one context's phase-2 sizing and warm-up)
            if (g_fake_devs) {
                if (g_fake_delay_us) usleep(g_fake_delay_us);
            } else {
                check(hipSetDevice(c->dev), "hipSetDevice");
                presize(c);
                warm(c);
            }
        } catch (const std::bad_alloc&) {
        }
        c->full = true;   // (also after an allocation failure: not tried again)
        pthread_mutex_lock(&g_pool_m);
        g_pool[g_pool_n++] = c;
        pthread_cond_broadcast(&g_pool_cv);
        pthread_mutex_unlock(&g_pool_m);
    }
    pthread_mutex_lock(&g_pool_m);
    g_pre_running = false;
    g_pre_phase1 = false;
    pthread_cond_broadcast(&g_pool_cv);
    pthread_mutex_unlock(&g_pool_m);
    return nullptr;
}
// Stops the start-up thread between two steps and waits for it.  Called from on_exit_handler, which
// init_once registers right after the runtime's first call, so it runs before any exit hook the
// runtime registered while starting up; preinit_exit (registered by the constructor) is the
// fallback for a process that exits before that.
void preinit_join() {
    g_pre_stop.store(true);
    if (g_pre_started.exchange(false)) pthread_join(g_pre_thread, nullptr);
}
void preinit_exit() { preinit_join(); }
// Whether the main program itself names this library among its DT_NEEDED entries (the reference
// server linked with -lrle_mi355x), as opposed to a process that dlopen()s it
// (Python's ctypes: tests, bench.py, the torch binding).  Only such a program gets the background
// start-up by default (loading the library from Python must not initialise the GPU, and
// a multi-rank job must not build contexts on every rank's GPUs).
int needed_by_main_cb(struct dl_phdr_info* info, size_t, void* out) {
    const ElfW(Dyn)* dyn = nullptr;
    for (int i = 0; i < info->dlpi_phnum; ++i)
        if (info->dlpi_phdr[i].p_type == PT_DYNAMIC)
            dyn = reinterpret_cast<const ElfW(Dyn)*>(info->dlpi_addr + info->dlpi_phdr[i].p_vaddr);
    if (dyn) {
        // the loader rewrites DT_STRTAB in place to an absolute address on x86-64; take the form that
        // lies inside one of the object's loaded segments
        uintptr_t strtab = 0;
        for (const ElfW(Dyn)* d = dyn; d->d_tag != DT_NULL; ++d)
            if (d->d_tag == DT_STRTAB) strtab = (uintptr_t)d->d_un.d_ptr;
        auto inside = [&](uintptr_t a) {
            for (int i = 0; i < info->dlpi_phnum; ++i) {
                const ElfW(Phdr)& ph = info->dlpi_phdr[i];
                const uintptr_t lo = info->dlpi_addr + ph.p_vaddr;
                if (ph.p_type == PT_LOAD && a >= lo && a < lo + ph.p_memsz) return true;
            }
            return false;
        };
        if (strtab && !inside(strtab)) strtab += info->dlpi_addr;
        if (strtab && inside(strtab))
            for (const ElfW(Dyn)* d = dyn; d->d_tag != DT_NULL; ++d)
                if (d->d_tag == DT_NEEDED && strstr(reinterpret_cast<const char*>(strtab + d->d_un.d_val), "librle_mi355x"))
                    *static_cast<int*>(out) = 1;
    }
    return 1;   // the first object reported is the main program: stop there
}
bool needed_by_main() {
    int found = 0;
    dl_iterate_phdr(needed_by_main_cb, &found);
    return found != 0;
}
// fork() while the start-up thread runs: the child has no such thread and no usable HIP state, so it
// starts with an empty pool and no start-up in progress (pool_take would otherwise wait on a phase
// that never ends).
void preinit_atfork_prepare() { pthread_mutex_lock(&g_pool_m); }
void preinit_atfork_parent() { pthread_mutex_unlock(&g_pool_m); }
void preinit_atfork_child() {
    g_pool_n = 0;
    g_pre_running = g_pre_phase1 = false;
    g_pre_started.store(false);
    g_pre_stop.store(true);
    pthread_mutex_unlock(&g_pool_m);
}
__attribute__((constructor)) void preinit_start() {
    if (const char* t = getenv("RLE_MI355X_TRACE"))
        if (*t) g_trace = static_cast<TraceRec*>(calloc(kTraceMax, sizeof(TraceRec)));
    const char* e = getenv("RLE_MI355X_PREINIT");
    const bool linked = needed_by_main();
    if (e ? atoi(e) <= 0 : !linked) return;
    pthread_atfork(preinit_atfork_prepare, preinit_atfork_parent, preinit_atfork_child);
    atexit(preinit_exit);
    pthread_mutex_lock(&g_pool_m);
    g_pre_running = g_pre_phase1 = true;
    if (pthread_create(&g_pre_thread, nullptr, preinit_main, nullptr) == 0) g_pre_started.store(true);
    else g_pre_running = g_pre_phase1 = false;
    // Round 5: the program's main() starts once phase 1 is done (the runtime up and every pooled
    // context ready for small calls), so a server opens its socket already warm: clients that
    // connect the moment the socket appears no longer wait for the HIP runtime's start-up (the
    // cold battery 3).  The process starts that much later instead (tools/e2e_compare.py
    // reports both servers' start-up).  Bounded: after RLE_MI355X_PREINIT_WAIT_MS (default 5000; 0 =
    // do not wait, round 4's behaviour) main() starts anyway and the thread goes on in the background.
    // Only where the library is among the main program's DT_NEEDED entries: a dlopen()ed
    // library's constructor runs under the loader lock, and a dlopen inside the HIP runtime's start-up
    // on the thread would wait for that lock while this constructor waits for the thread, until the
    // timeout; so a dlopen()ed library (RLE_MI355X_PREINIT > 0) starts the thread and returns.
    long wait_ms = linked ? 5000 : 0;
    if (const char* w = getenv("RLE_MI355X_PREINIT_WAIT_MS"))
        if (linked) wait_ms = atol(w);
    if (wait_ms > 0 && g_pre_started.load()) {
        timespec until;
        clock_gettime(CLOCK_REALTIME, &until);
        until.tv_sec += wait_ms / 1000;
        until.tv_nsec += (wait_ms % 1000) * 1000000L;
        if (until.tv_nsec >= 1000000000L) {
            until.tv_sec += 1;
            until.tv_nsec -= 1000000000L;
        }
        while (g_pre_phase1)
            if (pthread_cond_timedwait(&g_pool_cv, &g_pool_m, &until) != 0) break;   // (ETIMEDOUT)
    }
    pthread_mutex_unlock(&g_pool_m);
}
extern "C" int rle_mi355x_preinit_state(void) { return g_pre_started.load() ? 1 : 0; }
#if RLE_TEST_HOOKS
Ctx* ctx();   // below
// Test build only: this thread's context (taken from the pool or made), its device.
extern "C" int rle_test_touch_ctx(void) { return ctx()->dev; }
#endif
// A warm context from the pool, or nullptr (none left and the thread has finished).
Ctx* pool_take() {
    pthread_mutex_lock(&g_pool_m);
    while (g_pool_n == 0 && g_pre_phase1) pthread_cond_wait(&g_pool_cv, &g_pool_m);
    for (int i = 0; i + 1 < g_pool_n; ++i)   // a sized and warmed context first
        if (g_pool[i]->full) {
            Ctx* t = g_pool[i];
            g_pool[i] = g_pool[g_pool_n - 1];
            g_pool[g_pool_n - 1] = t;
            break;
        }
    Ctx* c = g_pool_n ? g_pool[--g_pool_n] : nullptr;
    pthread_mutex_unlock(&g_pool_m);
    return c;
}

Ctx* ctx() {
    pthread_once(&g_once, init_once);
    Ctx* c = static_cast<Ctx*>(pthread_getspecific(g_key));
    if (c) {
        if (!g_fake_devs) check(hipSetDevice(c->dev), "hipSetDevice");
        return c;
    }
    if (g_ndev <= 0) {
        fprintf(stderr, "librle_mi355x: no HIP device is visible; the RLE codec runs on MI355X only\n");
        abort();
    }
    const uint64_t t0 = g_trace ? now_ns() : 0;
    c = pool_take();
    if (c && !g_fake_devs) check(hipSetDevice(c->dev), "hipSetDevice");
    else c = new_ctx((g_dev_pin >= 0 && g_dev_pin < g_ndev) ? g_dev_pin : (int)(g_next_dev++ % (unsigned)g_ndev),
                     !g_pre_started.load());   // (beside the start-up thread: unsized, for a short first call)
    pthread_setspecific(g_key, c);
    if (g_trace) t_ctx_ns = now_ns() - t0;
    return c;
}

// After an allocation failure part of a call may still be queued on the thread's stream: let it
// finish before the next call reuses (or regrows) the buffers it refers to.
void drain_after_oom() {
    if (Ctx* c = static_cast<Ctx*>(pthread_getspecific(g_key))) (void)hipStreamSynchronize(c->s);
    errno = ENOMEM;
}

// Staging and device buffers grow on demand (never below 16 bytes, so a launch never sees NULL).
// A failed allocation throws std::bad_alloc, which each entry point turns into the reference's
// allocation-failure result (NULL, or -1 with errno = ENOMEM) instead of aborting the server.
void grow_host(uint8_t*& p, size_t& cap, size_t need) {
    need = std::max<size_t>(need, 16);
    if (need <= cap) return;
    size_t n = cap ? cap : (64u << 10);
    while (n < need) n *= 2;
    if (p) check(hipHostFree(p), "hipHostFree");
    p = nullptr;
    cap = 0;
    if (injected_failure(n) || hipHostMalloc(reinterpret_cast<void**>(&p), n, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        p = nullptr;
        throw std::bad_alloc();
    }
    cap = n;
}
void grow_dev(uint8_t*& p, size_t& cap, size_t need) {
    need = std::max<size_t>(need, 16);
    if (need <= cap) return;
    size_t n = cap ? cap : (64u << 10);
    while (n < need) n *= 2;
    if (p) check(hipFree(p), "hipFree");
    p = nullptr;
    cap = 0;
    if (injected_failure(n) || hipMalloc(reinterpret_cast<void**>(&p), n) != hipSuccess) {
        (void)hipGetLastError();
        p = nullptr;
        throw std::bad_alloc();
    }
    cap = n;
}


}  // namespace

namespace {

// An encode whose status is not OK has no trustworthy output (RLE_STATUS_INTERNAL: the segmented
// kernels' carry wait ran out; never expected): the call fails loudly rather than return it.
void check_encode_status(uint32_t st) {
    if (st != RLE_STATUS_OK) {
        fprintf(stderr, "librle_mi355x: RLEcompress: encode status 0x%x\n", st);
        abort();
    }
}

// Queues on c->s the encode of n device bytes at d_src (16-byte aligned) into c->d_out, the D2H of
// C into h_meta[kMetaEnc + 3] and, up to kOneTripBytes, of the worst-case output into h_out (one
// stream sync per call).  Returns whether the output travels with its size.
bool queue_encode(Ctx* c, const uint8_t* d_src, size_t n) {
    const size_t maxC = rle_max_compressed_size(n);
    grow_dev(c->d_out, c->d_out_cap, round16(maxC));
    uint64_t* hm = c->h_meta + kMetaEnc;
    uint64_t* dm = c->d_meta + kMetaEnc;
    hm[0] = 0; hm[1] = n; hm[2] = 0; hm[3] = 0;
    check(hipMemcpyAsync(dm, hm, 4 * sizeof(uint64_t), hipMemcpyHostToDevice, c->s), "H2D(meta)");
    uint32_t* d_status = reinterpret_cast<uint32_t*>(dm + 5);
    if (n >= kSegEncodeBytes) grow_dev(c->d_ws, c->d_ws_cap, rle_seg_workspace_bytes(1, n));
    const int erc = n >= kSegEncodeBytes
                        ? rle_encode_batch_device_seg(d_src, dm + 0, dm + 1, c->d_out, dm + 2, dm + 3, d_status, 1, n,
                                                      c->d_ws, c->d_ws_cap, c->s)
                        : rle_encode_batch_device_sized(d_src, dm + 0, dm + 1, c->d_out, dm + 2, dm + 3, d_status, 1, n, c->s);
    if (erc != RLE_OK) die("encode launch", hipGetLastError());
    check(hipMemcpyAsync(hm + 3, dm + 3, 3 * sizeof(uint64_t), hipMemcpyDeviceToHost, c->s), "D2H(meta)");
    const bool one_trip = n <= kOneTripBytes;
    if (one_trip) {
        grow_host(c->h_out, c->h_out_cap, maxC);
        check(hipMemcpyAsync(c->h_out, c->d_out, maxC, hipMemcpyDeviceToHost, c->s), "D2H");
    }
    return one_trip;
}

// After the stream sync that follows queue_encode: makes encoded bytes [from, C) present in h_out
// and returns C.
size_t fetch_encoded(Ctx* c, bool one_trip, size_t from) {
    const size_t C = c->h_meta[kMetaEnc + 3];
    check_encode_status((uint32_t)c->h_meta[kMetaEnc + 5]);
    if (!one_trip && C > from) {
        grow_host(c->h_out, c->h_out_cap, C);
        check(hipMemcpyAsync(c->h_out + from, c->d_out + from, C - from, hipMemcpyDeviceToHost, c->s), "D2H");
        check(hipStreamSynchronize(c->s), "hipStreamSynchronize");
    }
    return C;
}

// The caller's block: head[0, headLen) ‖ h_out[from, C) ‖ 16 zero bytes (the reference's calloc'd
// block ends in zeros that decoders read past C).  NULL on allocation failure; *outC always set.
char* make_block_from(const uint8_t* src, const char* head, size_t headLen, size_t from, size_t C, size_t* outC) {
    const size_t total = headLen + (C - from);
    *outC = total;
    char* r = static_cast<char*>(malloc(total + 16));
    if (!r) return nullptr;
    if (headLen) memcpy(r, head, headLen);
    memcpy(r + headLen, src + from, C - from);
    memset(r + total, 0, 16);
    return r;
}
char* make_block(const Ctx* c, const char* head, size_t headLen, size_t from, size_t C, size_t* outC) {
    return make_block_from(c->h_out, head, headLen, from, C, outC);
}

// Queues the decode of C device bytes at d_src into d_dst (U decoded bytes, slot of cap bytes) and
// the D2H of its status into h_meta[kMetaDec + 5].
void queue_decode(Ctx* c, const uint8_t* d_src, size_t C, uint8_t* d_dst, size_t U, size_t cap) {
    uint64_t* hm = c->h_meta + kMetaDec;
    uint64_t* dm = c->d_meta + kMetaDec;
    hm[0] = 0; hm[1] = C; hm[2] = 0; hm[3] = U; hm[4] = cap; hm[5] = 0;
    check(hipMemcpyAsync(dm, hm, 6 * sizeof(uint64_t), hipMemcpyHostToDevice, c->s), "H2D(meta)");
    uint32_t* d_status = reinterpret_cast<uint32_t*>(dm + 5);
    if (C >= kSegDecodeBytes) grow_dev(c->d_ws, c->d_ws_cap, rle_seg_workspace_bytes(1, C));
    const int drc = C >= kSegDecodeBytes
                        ? rle_decode_batch_device_seg(d_src, dm + 0, dm + 1, d_dst, dm + 2, dm + 3, dm + 4, d_status, 1,
                                                      C, c->d_ws, c->d_ws_cap, c->s)
                        : rle_decode_batch_device_sized(d_src, dm + 0, dm + 1, d_dst, dm + 2, dm + 3, dm + 4, d_status, 1,
                                                        C, U, c->s);
    if (drc != RLE_OK) die("decode launch", hipGetLastError());
    check(hipMemcpyAsync(hm + 5, dm + 5, sizeof(uint64_t), hipMemcpyDeviceToHost, c->s), "D2H(meta)");
}

void warn_overflow(const char* who) {
    if (!g_warned_overflow.exchange(1))
        fprintf(stderr, "librle_mi355x: %s: stream decodes past U+E (the reference would overflow its heap block); "
                        "output truncated\n", who);
}

// Chunk size of the pipelined transfers: at least 256 KiB, at most kPipeEvents chunks.
size_t pipe_chunk(size_t n) {
    size_t ch = 256u << 10;
    while ((n + ch - 1) / ch > (size_t)kPipeEvents) ch *= 2;
    return ch;
}

// Whether to_device copies n bytes through the pinned staging (else straight from the caller).
bool direct(const void* p, size_t n) {
    return g_staging == Staging::Direct && n >= kPipeMinBytes && !live_pages(p, n);
}
bool staged(const void* p, size_t n) { return n > 0 && !direct(p, n); }

// Queues the copy of n caller bytes at src to d_dst on c->s, staged (when staged) at h_in + hoff;
// src may be reused on return.  Callers queuing several copies grow h_in for all of them first.
void to_device(Ctx* c, uint8_t* d_dst, const void* src, size_t n, size_t hoff = 0) {
    const uint8_t* p = static_cast<const uint8_t*>(src);
    if (n == 0) return;
    if (direct(p, n)) {
        check(hipMemcpyAsync(d_dst, p, n, hipMemcpyHostToDevice, c->s), "H2D");
        return;
    }
    grow_host(c->h_in, c->h_in_cap, hoff + n);
    uint8_t* h = c->h_in + hoff;
    const size_t ch = (g_staging == Staging::Pipe && n >= kPipeMinBytes) ? pipe_chunk(n) : n;
    for (size_t off = 0; off < n; off += ch) {
        const size_t len = n - off < ch ? n - off : ch;
        memcpy(h + off, p + off, len);
        check(hipMemcpyAsync(d_dst + off, h + off, len, hipMemcpyHostToDevice, c->s), "H2D");
    }
}

// Copies n device bytes at d_src (after everything queued on c->s) into the caller's dst; returns
// with the stream drained up to that copy.
void from_device(Ctx* c, void* dst, const uint8_t* d_src, size_t n) {
    uint8_t* q = static_cast<uint8_t*>(dst);
    if (n == 0) {
        check(hipStreamSynchronize(c->s), "hipStreamSynchronize");
        return;
    }
    if (direct(q, n)) {
        check(hipMemcpyAsync(q, d_src, n, hipMemcpyDeviceToHost, c->s), "D2H");
        check(hipStreamSynchronize(c->s), "hipStreamSynchronize");
        return;
    }
    grow_host(c->h_out, c->h_out_cap, n);
    if (g_staging != Staging::Pipe || n < kPipeMinBytes) {
        check(hipMemcpyAsync(c->h_out, d_src, n, hipMemcpyDeviceToHost, c->s), "D2H");
        check(hipStreamSynchronize(c->s), "hipStreamSynchronize");
        memcpy(q, c->h_out, n);
        return;
    }
    const size_t ch = pipe_chunk(n);
    int k = 0;
    for (size_t off = 0; off < n; off += ch, ++k) {
        const size_t len = n - off < ch ? n - off : ch;
        if (!c->ev[k]) check(hipEventCreateWithFlags(&c->ev[k], hipEventDisableTiming), "hipEventCreate");
        check(hipMemcpyAsync(c->h_out + off, d_src + off, len, hipMemcpyDeviceToHost, c->s), "D2H");
        check(hipEventRecord(c->ev[k], c->s), "hipEventRecord");
    }
    k = 0;
    for (size_t off = 0; off < n; off += ch, ++k) {
        const size_t len = n - off < ch ? n - off : ch;
        check(hipEventSynchronize(c->ev[k]), "hipEventSynchronize");
        memcpy(q + off, c->h_out + off, len);
    }
}

// Small calls (one-wave kernels, output <= kOneTripBytes).  Zero-copy (default): the caller's bytes,
// the launch words and the result live in the thread's mapped pinned buffer (kZc* layout).  Copying
// (RLE_MI355X_SMALL=copy): the launch words travel inside the data copies -- the input words after
// the caller's bytes in the one H2D, the output length / status after the output slot in the one
// D2H -- so a call is one H2D, one launch, one D2H, one sync.
constexpr size_t kMetaBytes = 64;

uint8_t* zc(Ctx* c) {
    if (!c->h_zc) {
        if (hipHostMalloc(reinterpret_cast<void**>(&c->h_zc), kZcBytes, hipHostMallocMapped) != hipSuccess) {
            (void)hipGetLastError();
            c->h_zc = nullptr;
            throw std::bad_alloc();
        }
        check(hipHostGetDevicePointer(reinterpret_cast<void**>(&c->d_zc), c->h_zc, 0), "hipHostGetDevicePointer");
    }
    return c->h_zc;
}

// A new thread context gets its buffers at once: the zero-copy buffer and g_presize bytes of pinned
// staging and device buffers each way, so that the first medium-size calls do not pay pinned-memory
// growth (hipHostMalloc of a few hundred KiB costs milliseconds: r2i e2e, 7.6 ms of ns_stage_in for
// 883 KB).  RLE_MI355X_PRESIZE=<bytes> (0: grow lazily).  A failed allocation here is not an error:
// the buffers then grow on demand as before.
void presize(Ctx* c) {
    if (!g_presize) return;
    try {
        zc(c);
        grow_host(c->h_in, c->h_in_cap, g_presize);
        grow_host(c->h_out, c->h_out_cap, g_presize);
        grow_dev(c->d_in, c->d_in_cap, g_presize);
        grow_dev(c->d_out, c->d_out_cap, g_presize);
    } catch (const std::bad_alloc&) {
    }
}

#if RLE_VARIANTS
// ---------------------------------------------------------------- coalescing of concurrent small calls
// The server's worker threads (src/server.c:520-524) call the codec concurrently -- reads of
// different files decode outside the store lock (src/filesystemApi.c:570 -> 597) -- and a 4 KiB
// call is bound by its fixed cost (one launch, one sync: ~18 us), not by the GPU.  So concurrent
// zero-copy calls on one device join one batched launch (flat combining): each caller puts its
// bytes in its own mapped buffer and a request on the device's queue; whichever caller finds no
// batch in flight becomes the combiner, takes every queued request, issues one encode and/or one
// decode launch over all of them on its stream (the kernels read and write the callers' mapped
// buffers; offsets are relative to the lowest buffer address), syncs once and marks each request
// done.  Requests that arrive meanwhile wait for the next combiner.  A caller alone pays two mutex
// operations more than before.  Outputs are the same bytes: each buffer is independent
// (src/rleCompression.c:9-62).
// Off by default (RLE_MI355X_COALESCE=1 turns it on): measured with tools/callrate (4 KiB round
// trips, r3d), one stream per thread already overlaps the calls on the GPU's hardware queues --
// 55.8 K calls/s on 1 thread, 98.7 K on 2, 250.6 K on 8, 291.7 K on 16 -- while combining serialises
// them behind the batch in flight: 52.9 K, 145.2 K and 248.6 K calls/s on 2, 8 and 16 threads.
constexpr uint32_t kMaxCoalesce = 256;   // requests per combined launch
struct Req {
    const uint8_t* d_buf;   // the caller's mapped buffer (device address): input at kZcIn, output at kZcOut
    uint64_t in_len;        // encode: U; decode: C
    uint64_t out_len;       // decode: U
    uint64_t cap;           // decode: U + E
    bool dec;
    uint64_t result;        // encode: C; decode: status
    std::atomic<int> done{0};
};
struct Combiner {
    std::mutex m;
    std::vector<Req*> q;
    std::atomic<bool> busy{false};
};
constexpr int kMaxDev = 64;
Combiner g_comb[kMaxDev];

// Launch words of one combined launch in the combiner's mapped buffer: per kind 5 u64 arrays (in_off,
// in_len, out_off, out_len, out_cap) and the u32 statuses.
constexpr size_t kCwBytes = 2 * (5 + 1) * 8 * kMaxCoalesce;
uint64_t* cw(Ctx* c, uint64_t** dev) {
    if (!c->h_cw) {
        if (hipHostMalloc(reinterpret_cast<void**>(&c->h_cw), kCwBytes, hipHostMallocMapped) != hipSuccess) {
            (void)hipGetLastError();
            c->h_cw = nullptr;
            throw std::bad_alloc();
        }
        check(hipHostGetDevicePointer(reinterpret_cast<void**>(&c->d_cw), c->h_cw, 0), "hipHostGetDevicePointer");
    }
    *dev = reinterpret_cast<uint64_t*>(c->d_cw);
    return reinterpret_cast<uint64_t*>(c->h_cw);
}

// One combined launch per kind over reqs[0, m), on c's stream, one sync.
void run_batch(Ctx* c, Req* const* reqs, uint32_t m) {
    uint64_t* dw = nullptr;
    uint64_t* hw = cw(c, &dw);
    const uint8_t* base = reqs[0]->d_buf;
    for (uint32_t i = 1; i < m; ++i) base = std::min(base, reqs[i]->d_buf);
    for (int dec = 0; dec < 2; ++dec) {
        uint64_t* h = hw + (size_t)dec * (5 + 1) * kMaxCoalesce;   // 5 u64 arrays + room for the statuses
        uint64_t* d = dw + (size_t)dec * (5 + 1) * kMaxCoalesce;
        uint32_t k = 0;
        uint64_t max_in = 0, max_out = 0;
        for (uint32_t i = 0; i < m; ++i) {
            const Req* r = reqs[i];
            if (r->dec != (dec != 0)) continue;
            const uint64_t off = (uint64_t)(r->d_buf - base);
            h[k] = off + kZcIn;
            h[kMaxCoalesce + k] = r->in_len;
            h[2 * kMaxCoalesce + k] = off + kZcOut;
            h[3 * kMaxCoalesce + k] = r->out_len;
            h[4 * kMaxCoalesce + k] = r->cap;
            max_in = std::max(max_in, r->in_len);
            max_out = std::max(max_out, r->out_len);
            ++k;
        }
        if (!k) continue;
        uint32_t* dst = reinterpret_cast<uint32_t*>(d + 5 * kMaxCoalesce);
        uint8_t* obase = const_cast<uint8_t*>(base);
        const int rc = dec ? rle_decode_batch_device_sized(base, d, d + kMaxCoalesce, obase, d + 2 * kMaxCoalesce,
                                                           d + 3 * kMaxCoalesce, d + 4 * kMaxCoalesce, dst, k, max_in,
                                                           max_out, c->s)
                           : rle_encode_batch_device_sized(base, d, d + kMaxCoalesce, obase, d + 2 * kMaxCoalesce,
                                                           d + 3 * kMaxCoalesce, dst, k, max_in, c->s);
        if (rc != RLE_OK) die(dec ? "decode launch" : "encode launch", hipGetLastError());
    }
    check(hipStreamSynchronize(c->s), "hipStreamSynchronize");
    uint32_t ke = 0, kd = 0;
    for (uint32_t i = 0; i < m; ++i) {
        Req* r = reqs[i];
        if (r->dec) {
            const uint32_t* st = reinterpret_cast<const uint32_t*>(hw + (5 + 1) * kMaxCoalesce + 5 * kMaxCoalesce);
            r->result = st[kd++];
        } else {
            r->result = hw[3 * kMaxCoalesce + ke++];
        }
        r->done.store(1, std::memory_order_release);
    }
    g_stats.launches_coalesced++;
    g_stats.calls_coalesced += m;
}

// Queue r on the device's combiner and return once it is done (this thread may run the batch).
void submit(Ctx* c, Req* r) {
    Combiner& cb = g_comb[c->dev % kMaxDev];
    {
        std::lock_guard<std::mutex> g(cb.m);
        cb.q.push_back(r);
    }
    Req* batch[kMaxCoalesce];
    for (unsigned spin = 0; !r->done.load(std::memory_order_acquire); ++spin) {
        if (!cb.busy.load(std::memory_order_relaxed) && !cb.busy.exchange(true, std::memory_order_acquire)) {
            uint32_t m = 0;
            {
                std::lock_guard<std::mutex> g(cb.m);
                m = (uint32_t)std::min<size_t>(cb.q.size(), kMaxCoalesce);
                std::copy(cb.q.begin(), cb.q.begin() + m, batch);
                cb.q.erase(cb.q.begin(), cb.q.begin() + m);
            }
            if (m) {
                try {
                    run_batch(c, batch, m);
                } catch (...) {   // allocation failure of the launch words: every waiter must still finish
                    for (uint32_t i = 0; i < m; ++i) {
                        batch[i]->result = ~0ull;
                        batch[i]->done.store(1, std::memory_order_release);
                    }
                }
            }
            cb.busy.store(false, std::memory_order_release);
        } else if (spin > 64) {
            sched_yield();
        }
    }
    if (r->result == ~0ull) throw std::bad_alloc();
}

#endif  // RLE_VARIANTS

// Launch flags and completion wait of a zero-copy call (g_poll): the status word in the mapped
// buffer is preset to kPending and polled, spinning for kSpinNs, then yielding the core between
// reads.  Past kPollNs of polling (a box under load, a kernel fault) the stream is synchronized,
// which also reports a failed launch; every kPollSyncEvery polled calls it is synchronized anyway,
// so the runtime's record of completed launches stays short.
constexpr uint32_t kPending = 0xFFFFFFFFu;
constexpr uint64_t kPollNs = 2000000;
// (g_spin_ns, above: then the poll yields the core between reads)
constexpr uint32_t kPollSyncEvery = 32;
uint32_t zc_flags() { return g_poll ? RLE_LAUNCH_STATUS_FLAG : 0u; }
uint32_t zc_wait(Ctx* c, const uint64_t* status_word) {
    const volatile uint32_t* st = reinterpret_cast<const volatile uint32_t*>(status_word);
    if (g_poll) {
        uint64_t t0 = 0;
        bool yield = false;
        for (uint32_t i = 1;; ++i) {
            const uint32_t v = __atomic_load_n(st, __ATOMIC_ACQUIRE);
            if (v != kPending) {
                if (++c->polled >= kPollSyncEvery) {
                    c->polled = 0;
                    check(hipStreamSynchronize(c->s), "hipStreamSynchronize");
                }
                return v;
            }
            if ((i & 63u) == 0u) {
                const uint64_t t = now_ns();
                if (!t0) t0 = t;
                else if (t - t0 > kPollNs) break;
                else yield = t - t0 > g_spin_ns;
            }
            if (yield) sched_yield();   // a long call: leave the core to the server's other threads
            else __builtin_ia32_pause();
        }
    }
    c->polled = 0;
    check(hipStreamSynchronize(c->s), "hipStreamSynchronize");
    const uint32_t v = __atomic_load_n(st, __ATOMIC_ACQUIRE);
    if (g_poll && v == kPending) die("status never stored", hipErrorUnknown);
    return v;
}

// ---------------------------------------------------------------- resident small-call service
// Measured slower than the per-call launches at 8 threads and behind the server (DESIGN.md §6,
// profiles/r4r_callrate.txt, r4r_e2e_compare.json), so since round 5 it is built only into the
// RLE_VARIANTS test library (RLE_MI355X_SERVICE=1 there); the product library carries stubs.
#if RLE_VARIANTS
// (rle_service.h): one resident workgroup per thread context, on the context's own service stream,
// its mailbox in the context's mapped buffer.  g_svc_m guards the registry of contexts with a
// service, which process exit stops (svc_stop).
extern "C" int rle_service_launch(void* d_mail, const void* d_src, void* d_dst, uint32_t gen, uint32_t done,
                                  void* stream);
constexpr size_t kZcMail = kZcWords + 2048;   // the mailbox's offset in the mapped buffer (64-byte aligned)
constexpr int kSvcMax = 256;                  // contexts with a service at once (the rest launch per call)
pthread_mutex_t g_svc_m = PTHREAD_MUTEX_INITIALIZER;
Ctx* g_svc_ctx[kSvcMax];
int g_svc_n = 0;

// Whether context c serves its small calls through its resident service (set up on first use).
bool svc_on(Ctx* c) {
    if (c->svc != -2) return c->svc > 0;
    c->svc = -1;
    if (!g_service) return false;
    zc(c);
    pthread_mutex_lock(&g_svc_m);
    const bool room = g_svc_n < kSvcMax;
    if (room) g_svc_ctx[g_svc_n++] = c;
    pthread_mutex_unlock(&g_svc_m);
    if (!room) return false;
    // The service stream at the greatest priority: the runtime serves each priority from its own
    // hardware queues, so the resident workgroup never shares a queue with the contexts' normal
    // streams, whose dependent launches (a call's second kernel waits for its first) would otherwise
    // wait behind it until it idles out (tools/probes/queue_probe.hip).
    int prio_lo = 0, prio_hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
    if (hipStreamCreateWithPriority(&c->svc_s, hipStreamNonBlocking, prio_hi) != hipSuccess) {
        (void)hipGetLastError();
        c->svc_s = nullptr;
        return false;   // (stays registered: svc_stop skips a context without a stream)
    }
    c->svc_h = reinterpret_cast<rle::SvcMail*>(c->h_zc + kZcMail);
    c->svc_d = reinterpret_cast<rle::SvcMail*>(c->d_zc + kZcMail);
    memset(c->svc_h, 0, sizeof(rle::SvcMail));
    c->svc = 1;
    return true;
}
// A running service for c's request just posted: launch one when there is none or the last has ended
// (wait for that launch to complete first).
std::atomic<bool> g_svc_stopped{false};   // svc_stop ran: no service is launched again
bool svc_ensure(Ctx* c) {
    if (c->svc_gen && __atomic_load_n(&c->svc_h->a.gone, __ATOMIC_ACQUIRE) != c->svc_gen) return true;
    if (g_svc_stopped.load(std::memory_order_acquire)) return false;
    if (c->svc_gen) check(hipStreamSynchronize(c->svc_s), "hipStreamSynchronize(service)");
    const uint32_t done = __atomic_load_n(&c->svc_h->a.ack, __ATOMIC_ACQUIRE);
    if (rle_service_launch(c->svc_d, c->d_zc + kZcIn, c->d_zc + kZcOut, c->svc_gen + 1u, done, c->svc_s) != RLE_OK)
        die("service launch", hipGetLastError());
    ++c->svc_gen;
    return true;
}
// End c's service and wait for it (thread exit, process exit).
void svc_end(Ctx* c) {
    if (c->svc <= 0 || !c->svc_s) return;
    if (c->svc_gen) {
        __atomic_store_n(&c->svc_h->r.stop, 1u, __ATOMIC_RELEASE);
        (void)hipStreamSynchronize(c->svc_s);
    }
    (void)hipStreamDestroy(c->svc_s);
    c->svc_s = nullptr;
    c->svc = -1;
}
void svc_unregister(Ctx* c) {
    pthread_mutex_lock(&g_svc_m);
    for (int i = 0; i < g_svc_n; ++i)
        if (g_svc_ctx[i] == c) {
            g_svc_ctx[i] = g_svc_ctx[--g_svc_n];
            break;
        }
    pthread_mutex_unlock(&g_svc_m);
}
// At exit (on_exit_handler, before the runtime's teardown): every service ends.
void svc_stop() {
    g_svc_stopped.store(true, std::memory_order_release);
    pthread_mutex_lock(&g_svc_m);
    for (int i = 0; i < g_svc_n; ++i)
        if (g_svc_ctx[i]->svc > 0 && g_svc_ctx[i]->svc_gen) __atomic_store_n(&g_svc_ctx[i]->svc_h->r.stop, 1u, __ATOMIC_RELEASE);
    for (int i = 0; i < g_svc_n; ++i)
        if (g_svc_ctx[i]->svc > 0 && g_svc_ctx[i]->svc_gen) (void)hipStreamSynchronize(g_svc_ctx[i]->svc_s);
    pthread_mutex_unlock(&g_svc_m);
}
// One request on c's mapped buffer: returns the status, *res_len the encoded size.  The line is
// written with the sequence number last (tail, then req); the wait polls ack, checking every 256
// polls that the service has not ended before taking the request.  Once process exit has stopped
// the services (svc_stop) a request that finds its service gone is not served: kSvcStopped, and the
// caller takes the launch path (a relaunch would exit at once on the stop word).
constexpr uint32_t kSvcStopped = 0xFFFFFFFFu;
uint32_t svc_call(Ctx* c, uint32_t op, uint64_t in_len, uint64_t out_len, uint64_t cap, uint64_t* res_len) {
    rle::SvcReq* r = &c->svc_h->r;
    r->op = op;
    r->in_len = (uint32_t)in_len;
    r->out_len = (uint32_t)out_len;
    r->cap = (uint32_t)cap;
    r->flags = 1u;   // write-through stores (the output leaves the L2 at once)
    const uint32_t seq = ++c->svc_seq;
    __atomic_store_n(&r->tail, seq, __ATOMIC_RELEASE);
    __atomic_store_n(&r->req, seq, __ATOMIC_RELEASE);
    if (!svc_ensure(c)) return kSvcStopped;
    const uint64_t t0 = now_ns();
    bool yield = false;
    for (uint32_t i = 1;; ++i) {
        if (__atomic_load_n(&c->svc_h->a.ack, __ATOMIC_ACQUIRE) == seq) break;
        if ((i & 255u) == 0u) {
            if (!svc_ensure(c) && __atomic_load_n(&c->svc_h->a.ack, __ATOMIC_ACQUIRE) != seq) return kSvcStopped;
            const uint64_t t = now_ns() - t0;
            if (t > 10000000000ull) die("service request (10 s)", hipErrorUnknown);
            yield = t > g_spin_ns;
        }
        if (yield) sched_yield();
        else __builtin_ia32_pause();
    }
    if (res_len) *res_len = __atomic_load_n(&c->svc_h->a.res_len, __ATOMIC_ACQUIRE);
    return __atomic_load_n(&c->svc_h->a.status, __ATOMIC_ACQUIRE);
}

#else
constexpr uint32_t kSvcStopped = 0xFFFFFFFFu;
inline bool svc_on(Ctx*) { return false; }
inline uint32_t svc_call(Ctx*, uint32_t, uint64_t, uint64_t, uint64_t, uint64_t*) { return kSvcStopped; }
void svc_end(Ctx*) {}
void svc_unregister(Ctx*) {}
void svc_stop() {}
#endif  // RLE_VARIANTS (resident service)

}  // namespace

// One buffer with its sizes as kernel arguments (csrc/rle_coop.hip): 1 launched, 0 not qualifying
// (the batched entry points are used), < 0 a launch error.
extern "C" int rle_encode_coop_one(const void* src, void* dst, uint64_t U, uint64_t* d_out_len, uint32_t* d_status,
                                   uint32_t flags, void* stream);
extern "C" int rle_decode_coop_one(const void* src, void* dst, uint64_t C, uint64_t U, uint64_t cap,
                                   uint32_t* d_status, uint32_t flags, void* stream);

namespace {
char* compress_small_zc(Ctx* c, const char* data, size_t U, size_t* compressedSize) {
    uint8_t* h = zc(c);
    memcpy(h + kZcIn, data, U);
    size_t C;
    uint32_t st_svc = 0;
#if RLE_VARIANTS
    if (g_coalesce) {
        Req r;
        r.d_buf = c->d_zc; r.in_len = U; r.out_len = 0; r.cap = 0; r.dec = false; r.result = 0;
        submit(c, &r);
        C = r.result;
    } else
#endif
    if (g_zc_seg && U >= g_zc_seg && !(g_zc_coop && U <= rle::kCoopEncMaxBytes)) {   // segmented kernels
        uint64_t* hw = reinterpret_cast<uint64_t*>(h + kZcWords);
        hw[0] = kZcIn; hw[1] = U; hw[2] = 0; hw[3] = 0; hw[4] = 0;
        uint64_t* dw = reinterpret_cast<uint64_t*>(c->d_zc + kZcWords);
        grow_dev(c->d_ws, c->d_ws_cap, rle_seg_workspace_bytes(1, U));
        if (rle_encode_batch_device_seg(c->d_zc, dw + 0, dw + 1, c->d_zc + kZcOut, dw + 2, dw + 3,
                                        reinterpret_cast<uint32_t*>(dw + 4), 1, U, c->d_ws, c->d_ws_cap, c->s) != RLE_OK)
            die("encode launch", hipGetLastError());
        check(hipStreamSynchronize(c->s), "hipStreamSynchronize");
        check_encode_status((uint32_t)hw[4]);
        C = hw[3];
    } else if (uint64_t Cs = 0; svc_on(c) && (st_svc = svc_call(c, rle::kSvcEncode, U, 0, 0, &Cs)) != kSvcStopped) {
        check_encode_status(st_svc);
        C = Cs;
    } else {
        uint64_t* hw = reinterpret_cast<uint64_t*>(h + kZcWords);
        hw[0] = kZcIn; hw[1] = U; hw[2] = 0; hw[3] = 0; hw[4] = kPending;
        uint64_t* dw = reinterpret_cast<uint64_t*>(c->d_zc + kZcWords);
        // the sizes by value where the cooperative kernels take the buffer: its first loads do not
        // wait for the launch words to come over PCIe
        const int one = rle_encode_coop_one(c->d_zc + kZcIn, c->d_zc + kZcOut, U, dw + 3,
                                            reinterpret_cast<uint32_t*>(dw + 4), zc_flags(), c->s);
        if (one < 0) die("encode launch", hipGetLastError());
        if (one == 0 &&
            rle_encode_batch_device_sized_flags(c->d_zc, dw + 0, dw + 1, c->d_zc + kZcOut, dw + 2, dw + 3,
                                                reinterpret_cast<uint32_t*>(dw + 4), 1, U, zc_flags(), c->s) != RLE_OK)
            die("encode launch", hipGetLastError());
        check_encode_status(zc_wait(c, hw + 4));
        C = hw[3];
    }
    *compressedSize = C;
    char* r = static_cast<char*>(malloc(C + 16));
    if (!r) return nullptr;
    memcpy(r, h + kZcOut, C);
    memset(r + C, 0, 16);
    return r;
}

void decompress_small_zc(Ctx* c, const char* data, size_t C, size_t U, size_t E, char* r) {
    const size_t total = U + E;
    uint8_t* h = zc(c);
    memcpy(h + kZcIn, data, C);
    uint32_t st;
#if RLE_VARIANTS
    if (g_coalesce) {
        Req r;
        r.d_buf = c->d_zc; r.in_len = C; r.out_len = U; r.cap = total; r.dec = true; r.result = 0;
        submit(c, &r);
        st = (uint32_t)r.result;
    } else
#endif
    if (g_zc_seg && C >= g_zc_seg && !(g_zc_coop && C <= rle::kCoopDecMaxIn && U <= rle::kCoopDecUmax)) {   // segmented
        uint64_t* hw = reinterpret_cast<uint64_t*>(h + kZcWords);
        hw[0] = kZcIn; hw[1] = C; hw[2] = 0; hw[3] = U; hw[4] = total; hw[5] = 0;
        uint64_t* dw = reinterpret_cast<uint64_t*>(c->d_zc + kZcWords);
        grow_dev(c->d_ws, c->d_ws_cap, rle_seg_workspace_bytes(1, C));
        if (rle_decode_batch_device_seg(c->d_zc, dw + 0, dw + 1, c->d_zc + kZcOut, dw + 2, dw + 3, dw + 4,
                                        reinterpret_cast<uint32_t*>(dw + 5), 1, C, c->d_ws, c->d_ws_cap, c->s) != RLE_OK)
            die("decode launch", hipGetLastError());
        check(hipStreamSynchronize(c->s), "hipStreamSynchronize");
        st = (uint32_t)hw[5];
    } else if (svc_on(c) && (st = svc_call(c, rle::kSvcDecode, C, U, total, nullptr)) != kSvcStopped) {
    } else {
        uint64_t* hw = reinterpret_cast<uint64_t*>(h + kZcWords);
        hw[0] = kZcIn; hw[1] = C; hw[2] = 0; hw[3] = U; hw[4] = total; hw[5] = kPending;
        uint64_t* dw = reinterpret_cast<uint64_t*>(c->d_zc + kZcWords);
        const int one = rle_decode_coop_one(c->d_zc + kZcIn, c->d_zc + kZcOut, C, U, total,
                                            reinterpret_cast<uint32_t*>(dw + 5), zc_flags(), c->s);
        if (one < 0) die("decode launch", hipGetLastError());
        if (one == 0 &&
            rle_decode_batch_device_sized_flags(c->d_zc, dw + 0, dw + 1, c->d_zc + kZcOut, dw + 2, dw + 3, dw + 4,
                                                reinterpret_cast<uint32_t*>(dw + 5), 1, C, U, zc_flags(), c->s) != RLE_OK)
            die("decode launch", hipGetLastError());
        st = zc_wait(c, hw + 5);
    }
    memcpy(r, h + kZcOut, U);
    if (E) {
        if (st & RLE_STATUS_SERIAL) memcpy(r + U, h + kZcOut + U, E);
        else memset(r + U, 0, E);
    }
    if (st & RLE_STATUS_OVERFLOW) warn_overflow("RLEdecompress");
}

// RLEcompress of U <= kOneTripBytes bytes; returns the caller's block.
char* compress_small(Ctx* c, const char* data, size_t U, size_t* compressedSize) {
    if (g_zerocopy) return compress_small_zc(c, data, U, compressedSize);
    const size_t Ur = round16(U), maxC = rle_max_compressed_size(U), Cr = round16(maxC);
    grow_host(c->h_in, c->h_in_cap, Ur + kMetaBytes);
    grow_host(c->h_out, c->h_out_cap, Cr + kMetaBytes);
    grow_dev(c->d_in, c->d_in_cap, Ur + kMetaBytes);
    grow_dev(c->d_out, c->d_out_cap, Cr + kMetaBytes);
    memcpy(c->h_in, data, U);
    uint64_t* hm = reinterpret_cast<uint64_t*>(c->h_in + Ur);
    hm[0] = 0; hm[1] = U; hm[2] = 0;
    check(hipMemcpyAsync(c->d_in, c->h_in, Ur + kMetaBytes, hipMemcpyHostToDevice, c->s), "H2D");
    uint64_t* dm = reinterpret_cast<uint64_t*>(c->d_in + Ur);
    uint64_t* dmo = reinterpret_cast<uint64_t*>(c->d_out + Cr);   // [C, status]
    if (rle_encode_batch_device_sized(c->d_in, dm + 0, dm + 1, c->d_out, dm + 2, dmo, reinterpret_cast<uint32_t*>(dmo + 1),
                                      1, U, c->s) != RLE_OK)
        die("encode launch", hipGetLastError());
    check(hipMemcpyAsync(c->h_out, c->d_out, Cr + kMetaBytes, hipMemcpyDeviceToHost, c->s), "D2H");
    check(hipStreamSynchronize(c->s), "hipStreamSynchronize");
    const size_t C = reinterpret_cast<const uint64_t*>(c->h_out + Cr)[0];
    check_encode_status((uint32_t)reinterpret_cast<const uint64_t*>(c->h_out + Cr)[1]);
    return make_block(c, nullptr, 0, 0, C, compressedSize);
}

// RLEdecompress of C, U + E <= kOneTripBytes into the caller's block r (U + E bytes).
void decompress_small(Ctx* c, const char* data, size_t C, size_t U, size_t E, char* r) {
    if (g_zerocopy) return decompress_small_zc(c, data, C, U, E, r);
    const size_t total = U + E, Cr = round16(C), Tr = round16(total);
    grow_host(c->h_in, c->h_in_cap, Cr + kMetaBytes);
    grow_host(c->h_out, c->h_out_cap, Tr + kMetaBytes);
    grow_dev(c->d_in, c->d_in_cap, Cr + kMetaBytes);
    grow_dev(c->d_out, c->d_out_cap, Tr + kMetaBytes);
    memcpy(c->h_in, data, C);
    uint64_t* hm = reinterpret_cast<uint64_t*>(c->h_in + Cr);
    hm[0] = 0; hm[1] = C; hm[2] = 0; hm[3] = U; hm[4] = total;
    check(hipMemcpyAsync(c->d_in, c->h_in, Cr + kMetaBytes, hipMemcpyHostToDevice, c->s), "H2D");
    uint64_t* dm = reinterpret_cast<uint64_t*>(c->d_in + Cr);
    uint32_t* d_status = reinterpret_cast<uint32_t*>(c->d_out + Tr);
    if (rle_decode_batch_device_sized(c->d_in, dm + 0, dm + 1, c->d_out, dm + 2, dm + 3, dm + 4, d_status, 1, C, U, c->s) !=
        RLE_OK)
        die("decode launch", hipGetLastError());
    check(hipMemcpyAsync(c->h_out, c->d_out, Tr + kMetaBytes, hipMemcpyDeviceToHost, c->s), "D2H");
    check(hipStreamSynchronize(c->s), "hipStreamSynchronize");
    const uint32_t st = reinterpret_cast<const uint32_t*>(c->h_out + Tr)[0];
    memcpy(r, c->h_out, U);
    // the E region: zeros, unless a non-encoder stream wrote into it (it travelled with the rest)
    if (E) {
        if (st & RLE_STATUS_SERIAL) memcpy(r + U, c->h_out + U, E);
        else memset(r + U, 0, E);
    }
    if (st & RLE_STATUS_OVERFLOW) warn_overflow("RLEdecompress");
}

// One call of every form on a fresh context (preinit_main), so its first real call pays no first
// use: the zero-copy small calls (one-wave and cooperative kernels), a segmented encode + decode
// through the pinned staging, and the runtime's pageable-memory copies of large calls (direct
// staging), which set up the copy engines and the runtime's own staging buffers on first use.
// One small call each way (phase 1 of the start-up): the zero-copy buffer and the stream's first
// launches.
void warm_small(Ctx* c) {
    uint8_t buf[4096], back[4096];
    for (size_t i = 0; i < sizeof(buf); ++i) buf[i] = (uint8_t)(((i * 2654435761u) >> 13) & 3u);
    size_t C = 0;
    char* r = compress_small(c, reinterpret_cast<const char*>(buf), sizeof(buf), &C);
    if (!r) throw std::bad_alloc();
    decompress_small(c, r, C, sizeof(buf), 0, reinterpret_cast<char*>(back));
    free(r);
}
void warm(Ctx* c) {
    const LargeCall lc(c->s);   // (its own buffers; a registration elsewhere only stages its copies)
    constexpr size_t kBig = kPipeMinBytes + (64u << 10), kMed = 64u << 10, kSmall = 4096;
    std::vector<uint8_t> buf(kBig), back(kBig);
    for (size_t i = 0; i < kBig; ++i) buf[i] = (uint8_t)(((i * 2654435761u) >> 13) & 3u);   // short runs
    const char* b = reinterpret_cast<const char*>(buf.data());
    char* out = reinterpret_cast<char*>(back.data());
    size_t C = 0;
    for (size_t n : {(size_t)16, kSmall}) {
        char* r = compress_small(c, b, n, &C);
        if (!r) throw std::bad_alloc();
        decompress_small(c, r, C, n, 0, out);
        free(r);
    }
    grow_dev(c->d_in, c->d_in_cap, kBig);
    grow_dev(c->d_mid, c->d_mid_cap, kMed);
    to_device(c, c->d_in, b, kMed);
    const bool one_trip = queue_encode(c, c->d_in, kMed);
    check(hipStreamSynchronize(c->s), "hipStreamSynchronize");
    C = fetch_encoded(c, one_trip, 0);
    queue_decode(c, c->d_out, C, c->d_mid, kMed, kMed);
    from_device(c, out, c->d_mid, kMed);
    if (!live_pages(b, kBig) && !live_pages(out, kBig)) {
        check(hipMemcpyAsync(c->d_in, b, kBig, hipMemcpyHostToDevice, c->s), "H2D");
        check(hipMemcpyAsync(out, c->d_in, kBig, hipMemcpyDeviceToHost, c->s), "D2H");
    }
    check(hipStreamSynchronize(c->s), "hipStreamSynchronize");
}

}  // namespace

int rle_append_prepare_launch(const void* d_mid, uint64_t U, void* d_head, unsigned long long* d_start,
                              uint64_t* d_res, hipStream_t s);   // csrc/rle_fileops.hip
int rle_copy_len_launch(void* dst, const void* src, const uint64_t* d_len, uint64_t max_bytes,
                        hipStream_t s);                          // csrc/rle_kernels.hip
int rle_copy_in_launch(void* dst, const void* src, uint64_t n, hipStream_t s);   // csrc/rle_kernels.hip

namespace {
// A registered call's input: read by a copy kernel through its device address when it is 16-byte
// aligned (the kernels after it start sooner than after a DMA, rle_kernels.hip copy_in_kernel), the
// DMA otherwise.  (A/B) RLE_MI355X_REG_KREAD=0: always the DMA.
const bool g_reg_kread = [] {
    const char* e = getenv("RLE_MI355X_REG_KREAD");
    return e ? atoi(e) != 0 : true;
}();
void reg_input(Ctx* c, const LargeCall& lc, const char* data, size_t n) {
    if (g_reg_kread && rle_copy_in_launch(c->d_in, lc.d_in, n, c->s) == RLE_OK) return;
    check(hipMemcpyAsync(c->d_in, data, n, hipMemcpyHostToDevice, c->s), "H2D");
}
}  // namespace

namespace {
// RLEappend of a small file (old stream decoded by one wave, c^r ‖ new encoded by one wave, output
// within kOneTripBytes) in one H2D and one D2H:
//   d_in  = [old stream | splice head (16) | new bytes | launch words]
//   d_out = [re-encoded tail | result words: C', encode status, decode status, r, head (2)]
// Returns false (and leaves nothing but d_mid's decoded old content behind) when the final-token
// check fails and the caller must re-encode whole; *Ce / *r then are meaningless.
constexpr size_t kAppendWords = 16;
bool append_small(Ctx* c, const char* content, size_t C, size_t U, const char* add, size_t A, size_t* Ce,
                  size_t* r) {
    const size_t Cr = round16(C), Ar = round16(A), offW = Cr + 16 + Ar, inBytes = offW + 8 * kAppendWords;
    const size_t Er = round16(rle_max_compressed_size(16 + A)), outBytes = Er + 64;
    grow_host(c->h_in, c->h_in_cap, inBytes);
    grow_host(c->h_out, c->h_out_cap, outBytes);
    grow_dev(c->d_in, c->d_in_cap, inBytes);
    grow_dev(c->d_out, c->d_out_cap, outBytes);
    grow_dev(c->d_mid, c->d_mid_cap, round16(U + A));
    memcpy(c->h_in, content, C);
    if (A) memcpy(c->h_in + Cr + 16, add, A);
    uint64_t* hw = reinterpret_cast<uint64_t*>(c->h_in + offW);
    hw[0] = 0; hw[1] = C; hw[2] = 0; hw[3] = U; hw[4] = U;   // decode: in_off, in_len, out_off, out_len, cap
    hw[5] = Cr; hw[6] = 16 + A; hw[7] = 0;                  // encode: in_off, in_len, out_off
    hw[8] = 0;                                               // final-run start accumulator
    check(hipMemcpyAsync(c->d_in, c->h_in, inBytes, hipMemcpyHostToDevice, c->s), "H2D");
    uint64_t* dw = reinterpret_cast<uint64_t*>(c->d_in + offW);
    uint64_t* res = reinterpret_cast<uint64_t*>(c->d_out + Er);
    if (rle_decode_batch_device_sized(c->d_in, dw + 0, dw + 1, c->d_mid, dw + 2, dw + 3, dw + 4,
                                      reinterpret_cast<uint32_t*>(res + 2), 1, C, U, c->s) != RLE_OK)
        die("decode launch", hipGetLastError());
    if (rle_append_prepare_launch(c->d_mid, U, c->d_in + Cr, reinterpret_cast<unsigned long long*>(dw + 8), res + 3,
                                  c->s) != RLE_OK)
        die("append launch", hipGetLastError());
    if (rle_encode_batch_device_sized(c->d_in, dw + 5, dw + 6, c->d_out, dw + 7, res + 0, reinterpret_cast<uint32_t*>(res + 1),
                                      1, 16 + A, c->s) != RLE_OK)
        die("encode launch", hipGetLastError());
    check(hipMemcpyAsync(c->h_out, c->d_out, outBytes, hipMemcpyDeviceToHost, c->s), "D2H");
    check(hipStreamSynchronize(c->s), "hipStreamSynchronize");
    const uint64_t* hr = reinterpret_cast<const uint64_t*>(c->h_out + Er);
    const uint32_t st = (uint32_t)hr[2];
    const size_t rr = hr[3];
    check_encode_status((uint32_t)hr[1]);
    const uint8_t ch = reinterpret_cast<const uint8_t*>(hr + 4)[15];
    const uint8_t* y = reinterpret_cast<const uint8_t*>(content);
    const size_t tok = rr == 1 ? 1 : 3;
    bool ok = st == RLE_STATUS_OK && rr >= 1 && rr <= 9 && C >= tok && y[C - tok] == ch;
    if (ok && tok == 3) ok = y[C - 2] == ch && y[C - 1] == (uint8_t)('0' + rr);
    *Ce = hr[0];
    *r = rr;
    return ok;
}

// RLEappend of a small file, zero-copy (round 6; g_zerocopy): the reference's own composition
// (src/filesystemApi.c:766-775: decode with the new bytes' room, the new bytes at U, encode of the
// whole) run on this thread's mapped buffer, two launches and one poll, no copy commands:
//   mapped input  = the old stream, then (once the decode has read it) the new stream
//   mapped output = decode(old)[0, U) written by the decode ‖ the new bytes (placed beforehand)
// For a small file the splice (append_small) saves nothing: its three extra launches cost more
// than re-encoding a few KiB (r6x: 4 KiB 35.4 µs through the splice on the mapped buffer against
// 32.8 staged and 26.7 as two drop-in calls).  Exact for any stream, as the composition is the
// reference's: the decode stops at U (cap U) and the encode covers U + A.  zc_append_fits: what
// the cooperative or one-wave kernels take from mapped memory.
bool zc_append_fits(size_t C, size_t U, size_t A) {
    if (!g_zerocopy || C == 0) return false;
    const bool dec = C < kSegDecodeBytes || (g_zc_coop && C <= rle::kCoopDecMaxIn && U <= rle::kCoopDecUmax);
    const bool enc = U + A < kSegEncodeBytes || (g_zc_coop && U + A <= rle::kCoopEncMaxBytes);
    return dec && enc && C <= kZcWords && U + A <= kZcMaxOut && rle_max_compressed_size(U + A) <= kZcWords;
}
char* append_small_zc(Ctx* c, const char* content, size_t C, size_t U, const char* add, size_t A, size_t* Cn) {
    uint8_t* h = zc(c);
    memcpy(h + kZcIn, content, C);
    if (A) memcpy(h + kZcOut + U, add, A);
    uint64_t* hw = reinterpret_cast<uint64_t*>(h + kZcWords);
    uint64_t* dw = reinterpret_cast<uint64_t*>(c->d_zc + kZcWords);
    hw[0] = kZcIn; hw[1] = C; hw[2] = kZcOut; hw[3] = U; hw[4] = U; hw[5] = kPending;           // decode
    hw[6] = kZcOut; hw[7] = U + A; hw[8] = kZcIn; hw[9] = 0; hw[10] = kPending;                // encode
    // (the sizes by value where the cooperative kernels take them, as compress_small_zc)
    const int d1 = rle_decode_coop_one(c->d_zc + kZcIn, c->d_zc + kZcOut, C, U, U,
                                       reinterpret_cast<uint32_t*>(dw + 5), zc_flags(), c->s);
    if (d1 < 0 || (d1 == 0 && rle_decode_batch_device_sized_flags(c->d_zc, dw + 0, dw + 1, c->d_zc, dw + 2, dw + 3,
                                                                   dw + 4, reinterpret_cast<uint32_t*>(dw + 5), 1, C,
                                                                   U, zc_flags(), c->s) != RLE_OK))
        die("decode launch", hipGetLastError());
    const int e1 = rle_encode_coop_one(c->d_zc + kZcOut, c->d_zc + kZcIn, U + A, dw + 9,
                                       reinterpret_cast<uint32_t*>(dw + 10), zc_flags(), c->s);
    if (e1 < 0 || (e1 == 0 && rle_encode_batch_device_sized_flags(c->d_zc, dw + 6, dw + 7, c->d_zc, dw + 8, dw + 9,
                                                                   reinterpret_cast<uint32_t*>(dw + 10), 1, U + A,
                                                                   zc_flags(), c->s) != RLE_OK))
        die("encode launch", hipGetLastError());
    check_encode_status(zc_wait(c, hw + 10));
    const uint32_t st = __atomic_load_n(reinterpret_cast<const uint32_t*>(hw + 5), __ATOMIC_ACQUIRE);
    if (st & RLE_STATUS_OVERFLOW) warn_overflow("RLEappend");
    return make_block_from(h + kZcIn, nullptr, 0, 0, hw[9], Cn);
}
}  // namespace

namespace {
// RLEcompress past the zero-copy reach without registration: the caller's bytes by the runtime's
// pageable copy (or the pinned staging: live_pages), the tokens back once their count is known.
// Inside a LargeCall.
char* compress_large(Ctx* c, const char* data, size_t U, size_t* compressedSize) {
    grow_dev(c->d_in, c->d_in_cap, round16(U));
    const uint64_t t0 = now_ns();
    to_device(c, c->d_in, data, U);
    const uint64_t t1 = now_ns();
    const bool one_trip = queue_encode(c, c->d_in, U);
    check(hipStreamSynchronize(c->s), "hipStreamSynchronize");
    const uint64_t t2 = now_ns();
    const size_t C = c->h_meta[kMetaEnc + 3];
    char* r;
    if (one_trip) {
        r = make_block(c, nullptr, 0, 0, C, compressedSize);
    } else {   // the output travels now that C is known, straight into the caller's block
        *compressedSize = C;
        r = static_cast<char*>(malloc(C + 16));
        if (r) {
            from_device(c, r, c->d_out, C);
            memset(r + C, 0, 16);
        }
    }
    const uint64_t t3 = now_ns();
    g_stats.calls_compress++;
    g_stats.bytes_in += U;
    g_stats.bytes_out += C;
    g_stats.bytes_h2d += U;
    g_stats.bytes_d2h += one_trip ? rle_max_compressed_size(U) : C;
    g_stats.ns_stage_in += t1 - t0;
    g_stats.ns_device += t2 - t1;
    g_stats.ns_stage_out += t3 - t2;
    return r;
}

// Whether an encode of n bytes takes the registered path (g_reg_min; the cooperative kernel's calls
// stay zero-copy).
bool registered_encode(size_t n) {
    return g_reg_min && !g_fake_devs && n >= g_reg_min && n >= kSegEncodeBytes &&
           !(g_zc_coop && n <= rle::kCoopEncMaxBytes);
}

// RLEcompress through registered memory (lc registered the caller's U bytes and the result block r
// of maxC + 16 bytes): the input DMA'd straight from the caller's pages, the tokens copied from
// device memory into r by the copy kernel, which reads their count on the device.  The device
// buffers are grown beforehand (compress_impl), so nothing here throws.
char* compress_registered(Ctx* c, const LargeCall& lc, const char* data, size_t U, char* r, size_t maxC,
                          size_t* compressedSize) {
    const uint64_t t0 = now_ns();
    // launch words in the thread's mapped buffer (as the zero-copy calls'): no copy commands for them,
    // so the stream is one DMA and four kernels
    uint64_t* hw = reinterpret_cast<uint64_t*>(c->h_zc + kZcWords);
    uint64_t* dw = reinterpret_cast<uint64_t*>(c->d_zc + kZcWords);
    hw[0] = 0; hw[1] = U; hw[2] = 0; hw[3] = 0; hw[4] = 0;
    reg_input(c, lc, data, U);
    if (rle_encode_batch_device_seg(c->d_in, dw + 0, dw + 1, c->d_out, dw + 2, dw + 3, reinterpret_cast<uint32_t*>(dw + 4),
                                    1, U, c->d_ws, c->d_ws_cap, c->s) != RLE_OK)
        die("encode launch", hipGetLastError());
    if (rle_copy_len_launch(lc.d_out, c->d_out, dw + 3, maxC, c->s) != RLE_OK) die("copy launch", hipGetLastError());
    check(hipStreamSynchronize(c->s), "hipStreamSynchronize");
    const size_t C = hw[3];
    check_encode_status((uint32_t)hw[4]);
    // The block keeps its worst-case size (the reference's own block is calloc(2U),
    // src/rleCompression.c:10): shrinking it in place returns the tail to malloc, whose next
    // worst-case block then comes fresh from the kernel each call (r6l: 1 MiB 521 against 87 µs).
    memset(r + C, 0, 16);
    *compressedSize = C;
    g_stats.calls_registered++;
    g_stats.calls_compress++;
    g_stats.bytes_in += U;
    g_stats.bytes_out += C;
    g_stats.bytes_h2d += U;
    g_stats.bytes_d2h += C;
    g_stats.ns_device += now_ns() - t0;
    return r;
}
}  // namespace

static char* compress_impl(char* data, size_t U, size_t* compressedSize) {
    Ctx* c = ctx();
    const bool reg = registered_encode(U) && reg_likely();
    const bool small = U < kSegEncodeBytes || (g_zc_seg && g_zerocopy && U <= kZcMaxIn);
    if (reg) {   // the registered path's buffers, grown before anything is registered
        const size_t maxC = rle_max_compressed_size(U);
        zc(c);
        grow_dev(c->d_in, c->d_in_cap, round16(U));
        grow_dev(c->d_out, c->d_out_cap, round16(maxC));
        grow_dev(c->d_ws, c->d_ws_cap, rle_seg_workspace_bytes(1, U));
        char* r = static_cast<char*>(malloc(maxC + 16));
        if (!r) throw std::bad_alloc();
        const LargeCall lc(c->s, data, U, r, maxC);
        if (lc.registered()) return compress_registered(c, lc, data, U, r, maxC, compressedSize);
        free(r);
        g_stats.calls_reg_fallback++;
        if (!small) return compress_large(c, data, U, compressedSize);
    } else if (!small) {
        const LargeCall lc(c->s);
        return compress_large(c, data, U, compressedSize);
    }
    // one wave walks it, or (g_zc_seg) the segmented kernels on the mapped buffer: the single-copy path
    const uint64_t t0 = now_ns();
    char* r = compress_small(c, data, U, compressedSize);
    g_stats.calls_compress++;
    g_stats.bytes_in += U;
    g_stats.bytes_out += *compressedSize;
    g_stats.bytes_h2d += round16(U) + kMetaBytes;
    g_stats.bytes_d2h += round16(rle_max_compressed_size(U)) + kMetaBytes;
    g_stats.ns_device += now_ns() - t0;
    return r;
}

// src/rleCompression.c:9-45 — returns a malloc block: C token bytes + >= 2 zero bytes; NULL (errno
// = ENOMEM) when an allocation fails, as the reference's calloc can (:10).
extern "C" char* RLEcompress(char* data, size_t origSize, size_t* compressedSize) {
    const size_t U = origSize;
    TraceScope ts('c', U, 0, 0);
    if (U == 0 || too_big("RLEcompress", U)) {
        *compressedSize = 0;
        return U == 0 ? static_cast<char*>(calloc(16, 1)) : nullptr;
    }
    try {
        return compress_impl(data, U, compressedSize);
    } catch (const std::bad_alloc&) {
        drain_after_oom();
        *compressedSize = 0;
        return nullptr;
    }
}

namespace {
// RLEdecompress through registered memory (as compress_registered; lc registered the caller's C
// bytes and the result block r of U + E bytes): the decoded bytes copied from device memory into r,
// and for a stream the encoder cannot have written, whatever it put into the E region.
void decompress_registered(Ctx* c, const LargeCall& lc, const char* data, size_t C, size_t U, size_t E, char* r) {
    const size_t total = U + E;
    const uint64_t t0 = now_ns();
    uint64_t* hw = reinterpret_cast<uint64_t*>(c->h_zc + kZcWords);   // (launch words: compress_registered)
    uint64_t* dw = reinterpret_cast<uint64_t*>(c->d_zc + kZcWords);
    hw[0] = 0; hw[1] = C; hw[2] = 0; hw[3] = U; hw[4] = total; hw[5] = 0;
    reg_input(c, lc, data, C);
    uint32_t* d_status = reinterpret_cast<uint32_t*>(dw + 5);
    const int drc = C >= kSegDecodeBytes
                        ? rle_decode_batch_device_seg(c->d_in, dw + 0, dw + 1, c->d_out, dw + 2, dw + 3, dw + 4, d_status,
                                                      1, C, c->d_ws, c->d_ws_cap, c->s)
                        : rle_decode_batch_device_sized(c->d_in, dw + 0, dw + 1, c->d_out, dw + 2, dw + 3, dw + 4,
                                                        d_status, 1, C, U, c->s);
    if (drc != RLE_OK) die("decode launch", hipGetLastError());
    if (rle_copy_len_launch(lc.d_out, c->d_out, dw + 3, U, c->s) != RLE_OK) die("copy launch", hipGetLastError());
    check(hipStreamSynchronize(c->s), "hipStreamSynchronize");
    const uint32_t st = (uint32_t)hw[5];
    if (E && (st & RLE_STATUS_SERIAL)) {   // a stream the encoder cannot have written may have put bytes
        // into the E region: they travel too (rare; one more round trip, inside r's registration)
        check(hipMemcpyAsync(r + U, c->d_out + U, E, hipMemcpyDeviceToHost, c->s), "D2H");
        check(hipStreamSynchronize(c->s), "hipStreamSynchronize");
    } else if (E) {
        memset(r + U, 0, E);
    }
    if (st & RLE_STATUS_OVERFLOW) warn_overflow("RLEdecompress");
    g_stats.calls_registered++;
    g_stats.calls_decompress++;
    g_stats.bytes_in += C;
    g_stats.bytes_out += total;
    g_stats.bytes_h2d += C;
    g_stats.bytes_d2h += U;
    g_stats.ns_device += now_ns() - t0;
}

// RLEdecompress past the zero-copy reach without registration (as compress_large).  Inside a
// LargeCall.
void decompress_large(Ctx* c, const char* data, size_t C, size_t U, size_t E, char* r);   // below
}  // namespace

static void decompress_impl(char* data, size_t C, size_t U, size_t E, char* r) {
    const size_t total = U + E;
    Ctx* c = ctx();
    const bool reg = g_reg_min && !g_fake_devs && (C >= g_reg_min || total >= g_reg_min) &&
                     !(g_zc_coop && C <= rle::kCoopDecMaxIn && U <= rle::kCoopDecUmax) && reg_likely();
    const bool small = (C < kSegDecodeBytes && total <= kOneTripBytes) ||
                       (g_zc_seg && g_zerocopy && C <= kZcMaxIn && total <= kZcMaxOut);
    if (reg) {   // the registered path's buffers, grown before anything is registered
        zc(c);
        grow_dev(c->d_in, c->d_in_cap, round16(C));
        grow_dev(c->d_out, c->d_out_cap, round16(total));
        if (C >= kSegDecodeBytes) grow_dev(c->d_ws, c->d_ws_cap, rle_seg_workspace_bytes(1, C));
        const LargeCall lc(c->s, data, C, r, total);
        if (lc.registered()) return decompress_registered(c, lc, data, C, U, E, r);
        g_stats.calls_reg_fallback++;
        if (!small) return decompress_large(c, data, C, U, E, r);
    } else if (!small) {
        const LargeCall lc(c->s);
        return decompress_large(c, data, C, U, E, r);
    }
    // one wave walks it, or (g_zc_seg) the segmented kernels on the mapped buffer: the single-copy path
    const uint64_t t0 = now_ns();
    decompress_small(c, data, C, U, E, r);
    g_stats.calls_decompress++;
    g_stats.bytes_in += C;
    g_stats.bytes_out += total;
    g_stats.bytes_h2d += round16(C) + kMetaBytes;
    g_stats.bytes_d2h += round16(total) + kMetaBytes;
    g_stats.ns_device += now_ns() - t0;
}

namespace {
void decompress_large(Ctx* c, const char* data, size_t C, size_t U, size_t E, char* r) {
    const size_t total = U + E;
    grow_dev(c->d_in, c->d_in_cap, round16(C));
    grow_dev(c->d_out, c->d_out_cap, round16(total));
    const uint64_t t0 = now_ns();
    to_device(c, c->d_in, data, C);
    const uint64_t t1 = now_ns();
    queue_decode(c, c->d_in, C, c->d_out, U, total);
    from_device(c, r, c->d_out, U);   // also completes the status copy queued before it
    const uint32_t st = (uint32_t)c->h_meta[kMetaDec + 5];
    const uint64_t t2 = now_ns();
    if (E) {
        if (st & RLE_STATUS_SERIAL) {  // a non-encoder stream may have written into the E region
            grow_host(c->h_out, c->h_out_cap, E);
            check(hipMemcpyAsync(c->h_out, c->d_out + U, E, hipMemcpyDeviceToHost, c->s), "D2H");
            check(hipStreamSynchronize(c->s), "hipStreamSynchronize");
            memcpy(r + U, c->h_out, E);
        } else {
            memset(r + U, 0, E);
        }
    }
    if (st & RLE_STATUS_OVERFLOW) warn_overflow("RLEdecompress");
    const uint64_t t3 = now_ns();
    g_stats.calls_decompress++;
    g_stats.bytes_in += C;
    g_stats.bytes_out += total;
    g_stats.bytes_h2d += C;
    g_stats.bytes_d2h += U;
    g_stats.ns_stage_in += t1 - t0;
    g_stats.ns_device += t2 - t1;
    g_stats.ns_stage_out += t3 - t2;
}
}  // namespace

// src/rleCompression.c:47-62 — returns a malloc block of U+E bytes (decoded U, then E zeros); NULL
// (errno = ENOMEM) when an allocation fails, as the reference's calloc can (:48).
extern "C" char* RLEdecompress(char* data, size_t compressedSize, size_t uncompressedSize, size_t extraAllocation) {
    const size_t C = compressedSize, U = uncompressedSize, E = extraAllocation, total = U + E;
    TraceScope ts('d', C, U, E);
    if (too_big("RLEdecompress", C) || too_big("RLEdecompress", U)) return nullptr;
    char* r = static_cast<char*>(malloc(total ? total : 1));
    if (!r) return nullptr;
    if (C == 0) {  // nothing to decode: calloc'd block (:48)
        memset(r, 0, total);
        return r;
    }
    try {
        decompress_impl(data, C, U, E, r);
        return r;
    } catch (const std::bad_alloc&) {
        drain_after_oom();
        free(r);
        return nullptr;
    }
}

// src/filesystemApi.c:766-775 (decode, append, re-encode) fused into one device
// round trip whose re-encode covers only c^r ‖ newContent (include/rle_fileops.h).
static char* append_impl(char* content, size_t C, size_t U, const char* newContent, size_t A,
                         size_t* newCompressedSize) {
    Ctx* c = ctx();
    if (zc_append_fits(C, U, A)) {   // zero-copy (append_small_zc)
        const uint64_t t0 = now_ns();
        char* out = append_small_zc(c, content, C, U, newContent, A, newCompressedSize);
        g_stats.calls_append++;
        g_stats.bytes_in += C + A;
        g_stats.bytes_out += *newCompressedSize;
        g_stats.bytes_h2d += C + A;
        g_stats.bytes_d2h += *newCompressedSize;
        g_stats.ns_device += now_ns() - t0;
        return out;
    }
    if (C && C < kSegDecodeBytes && 16 + A < kSegEncodeBytes &&
        rle_max_compressed_size(16 + A) <= kOneTripBytes) {
        const uint64_t t0 = now_ns();
        size_t Ce = 0, r = 0;
        char* out = nullptr;
        if (append_small(c, content, C, U, newContent, A, &Ce, &r)) {
            const size_t skip = 16 - r;
            out = make_block(c, content, C - (r == 1 ? 1 : 3), skip, Ce, newCompressedSize);
        } else {   // not encoder output: re-encode decode(old) ‖ new whole, as the reference does
            if (A) check(hipMemcpyAsync(c->d_mid + U, c->d_in + round16(C) + 16, A, hipMemcpyDeviceToDevice, c->s),
                         "D2D");
            const bool one_trip = queue_encode(c, c->d_mid, U + A);
            check(hipStreamSynchronize(c->s), "hipStreamSynchronize");
            const size_t Cn = fetch_encoded(c, one_trip, 0);
            out = make_block(c, nullptr, 0, 0, Cn, newCompressedSize);
        }
        g_stats.calls_append++;
        g_stats.bytes_in += C + A;
        g_stats.bytes_out += *newCompressedSize;
        g_stats.bytes_h2d += round16(C) + 16 + round16(A) + 8 * kAppendWords;
        g_stats.bytes_d2h += round16(rle_max_compressed_size(16 + A)) + 64;
        g_stats.ns_device += now_ns() - t0;
        return out;
    }
    const LargeCall lc(c->s);
    const size_t offA = round16(C) + 16;   // d_in: old stream | splice head (16 B) | new bytes
    const size_t inBytes = offA + A;
    // pinned staging only for the copies to_device stages (both, before either is queued)
    grow_host(c->h_in, c->h_in_cap, std::max(staged(newContent, A) ? inBytes : 0, staged(content, C) ? C : 0));
    grow_dev(c->d_in, c->d_in_cap, round16(inBytes));
    grow_dev(c->d_mid, c->d_mid_cap, round16(U + A));
    const uint64_t t0 = now_ns();
    to_device(c, c->d_in, content, C, 0);
    to_device(c, c->d_in + offA, newContent, A, offA);
    const uint64_t t1 = now_ns();
    bool full = C == 0;   // no stream: the decoded content is U zero bytes (:48), re-encoded whole
    bool one_trip = false;
    if (full) {
        check(hipMemsetAsync(c->d_mid, 0, U, c->s), "hipMemsetAsync");
    } else {
        queue_decode(c, c->d_in, C, c->d_mid, U, U);
        if (rle_append_prepare_device(c->d_mid, U, c->d_in + offA - 16, c->d_meta + kMetaApp, c->s) != RLE_OK)
            die("append launch", hipGetLastError());
        check(hipMemcpyAsync(c->h_meta + kMetaApp, c->d_meta + kMetaApp, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost,
                             c->s), "D2H(meta)");
        one_trip = queue_encode(c, c->d_in + offA - 16, 16 + A);
    }
    check(hipStreamSynchronize(c->s), "hipStreamSynchronize");
    size_t r = 0, tok = 0;
    if (!full) {
        // keep content[0, C - tok) only if the stream's final token is the one the encoder emits
        // for the decoded tail c^r (and the decode saw encoder output)
        const uint32_t st = (uint32_t)c->h_meta[kMetaDec + 5];
        r = c->h_meta[kMetaApp + 1];
        const uint8_t ch = reinterpret_cast<const uint8_t*>(c->h_meta + kMetaApp + 2)[15];
        const uint8_t* y = reinterpret_cast<const uint8_t*>(content);
        tok = r == 1 ? 1 : 3;
        bool ok = st == RLE_STATUS_OK && r >= 1 && r <= 9 && C >= tok && y[C - tok] == ch;
        if (ok && tok == 3) ok = y[C - 2] == ch && y[C - 1] == (uint8_t)('0' + r);
        full = !ok;
    }
    char* out;
    size_t Cn;
    if (full) {
        if (A) check(hipMemcpyAsync(c->d_mid + U, c->d_in + offA, A, hipMemcpyDeviceToDevice, c->s), "D2D");
        one_trip = queue_encode(c, c->d_mid, U + A);
        check(hipStreamSynchronize(c->s), "hipStreamSynchronize");
        Cn = fetch_encoded(c, one_trip, 0);
        out = make_block(c, nullptr, 0, 0, Cn, newCompressedSize);
    } else {
        const size_t skip = 16 - r;   // the filler's single-byte tokens
        Cn = fetch_encoded(c, one_trip, skip);
        out = make_block(c, content, C - tok, skip, Cn, newCompressedSize);
    }
    const uint64_t t2 = now_ns();
    g_stats.calls_append++;
    g_stats.bytes_in += C + A;
    g_stats.bytes_out += *newCompressedSize;
    g_stats.bytes_h2d += C + A;
    g_stats.bytes_d2h += full ? Cn : Cn - (16 - r);
    g_stats.ns_stage_in += t1 - t0;
    g_stats.ns_device += t2 - t1;
    return out;
}

extern "C" char* RLEappend(char* content, size_t contentSize, size_t uncompressedSize, const char* newContent,
                           size_t newContentLen, size_t* newCompressedSize) {
    const size_t C = contentSize, U = uncompressedSize, A = newContentLen;
    TraceScope ts('a', C, U, A);
    // U == 0: the decode keeps nothing below U and whatever it writes into the extra region is
    // overwritten by the appended bytes (:767-770), so the result is encode(newContent)
    if (U == 0) return RLEcompress(const_cast<char*>(newContent), A, newCompressedSize);
    if (too_big("RLEappend", C) || too_big("RLEappend", U + A)) {
        *newCompressedSize = 0;
        return nullptr;
    }
    try {
        return append_impl(content, C, U, newContent, A, newCompressedSize);
    } catch (const std::bad_alloc&) {
        drain_after_oom();
        *newCompressedSize = 0;
        return nullptr;
    }
}

namespace {
struct NTotals {
    size_t cin = 0, uout = 0, h2d = 0, d2h = 0;
    uint64_t ns_in = 0, ns_dev = 0, ns_out = 0;
};

// RLEdecompressN of one file too large for the bounded staging: straight from / to caller memory
// whatever RLE_MI355X_STAGING says (the pinned and pipe modes would grow this thread's staging to
// the file's size, which g_stage_cap exists to prevent).
// Bytes whose pages meet another call's registration (live_pages) go through the staging in
// chunks of at most g_stage_cap instead, a synchronize per chunk.
void decompress_n_alone(Ctx* c, const char* data, size_t C, size_t U, char* out, NTotals& t) {
    const LargeCall lc(c->s);
    grow_dev(c->d_in, c->d_in_cap, round16(C));
    grow_dev(c->d_out, c->d_out_cap, round16(U));
    const size_t ch = std::min(g_stage_cap, std::max(C, U));
    const bool stage_in = live_pages(data, C), stage_out = U && live_pages(out, U);
    if (stage_in) grow_host(c->h_in, c->h_in_cap, ch);
    if (stage_out) grow_host(c->h_out, c->h_out_cap, ch);
    const uint64_t t0 = now_ns();
    if (!stage_in) {
        check(hipMemcpyAsync(c->d_in, data, C, hipMemcpyHostToDevice, c->s), "H2D");
    } else {
        for (size_t off = 0; off < C; off += ch) {
            const size_t len = std::min(ch, C - off);
            memcpy(c->h_in, data + off, len);
            check(hipMemcpyAsync(c->d_in + off, c->h_in, len, hipMemcpyHostToDevice, c->s), "H2D");
            check(hipStreamSynchronize(c->s), "hipStreamSynchronize");
        }
    }
    const uint64_t t1 = now_ns();
    queue_decode(c, c->d_in, C, c->d_out, U, U);
    if (!stage_out) {
        if (U) check(hipMemcpyAsync(out, c->d_out, U, hipMemcpyDeviceToHost, c->s), "D2H");
        check(hipStreamSynchronize(c->s), "hipStreamSynchronize");
    } else {
        check(hipStreamSynchronize(c->s), "hipStreamSynchronize");
        for (size_t off = 0; off < U; off += ch) {
            const size_t len = std::min(ch, U - off);
            check(hipMemcpyAsync(c->h_out, c->d_out + off, len, hipMemcpyDeviceToHost, c->s), "D2H");
            check(hipStreamSynchronize(c->s), "hipStreamSynchronize");
            memcpy(out + off, c->h_out, len);
        }
    }
    if ((uint32_t)c->h_meta[kMetaDec + 5] & RLE_STATUS_OVERFLOW) warn_overflow("RLEdecompressN");
    t.ns_in += t1 - t0;
    t.ns_dev += now_ns() - t1;
    t.h2d += C;
    t.d2h += U;
}

// RLEdecompressN of the files idx[0, m) (each C > 0), staged together: one H2D, one launch per
// kernel form, one D2H.  Their staged sizes sum to at most g_stage_cap each way.
void decompress_n_chunk(Ctx* c, size_t* idx, size_t m, char* const* data, const size_t* compressedSize,
                        const size_t* uncompressedSize, char* const* out, NTotals& t) {
    size_t inTot = 0, outTot = 0, maxC = 0;
    for (size_t k = 0; k < m; ++k) {
        inTot += round16(compressedSize[idx[k]]);
        outTot += round16(uncompressedSize[idx[k]]);
        maxC = std::max(maxC, compressedSize[idx[k]]);
    }
    // files from kSegDecodeBytes up go to the segmented form, the rest to the one-wave kernel: the
    // large ones are packed first so that each launch takes a contiguous part of the metadata
    const size_t mL = maxC >= kSegDecodeBytes
                          ? (size_t)(std::stable_partition(idx, idx + m,
                                                           [&](size_t i) { return compressedSize[i] >= kSegDecodeBytes; }) -
                                     idx)
                          : 0;
    size_t inLarge = 0, maxCs = 0, maxUs = 0;
    for (size_t k = 0; k < mL; ++k) inLarge += round16(compressedSize[idx[k]]);
    for (size_t k = mL; k < m; ++k) {   // the one-wave launch's sizes (the cooperative kernels' hint)
        maxCs = std::max(maxCs, compressedSize[idx[k]]);
        maxUs = std::max(maxUs, uncompressedSize[idx[k]]);
    }
    // per-file metadata, one pinned block: in_off, in_len, out_off, out_len (m u64 each), status (m u32)
    const size_t metaBytes = 32 * m + 4 * m;
    grow_host(c->h_bm, c->h_bm_cap, metaBytes);
    grow_dev(c->d_bm, c->d_bm_cap, round16(metaBytes));
    grow_host(c->h_in, c->h_in_cap, inTot);
    grow_host(c->h_out, c->h_out_cap, outTot);
    grow_dev(c->d_in, c->d_in_cap, inTot);
    grow_dev(c->d_out, c->d_out_cap, outTot);
    if (mL) grow_dev(c->d_ws, c->d_ws_cap, rle_seg_workspace_bytes((uint32_t)mL, inLarge));
    const uint64_t t0 = now_ns();
    uint64_t* hb = reinterpret_cast<uint64_t*>(c->h_bm);
    size_t io = 0, oo = 0;
    for (size_t k = 0; k < m; ++k) {
        const size_t i = idx[k], C = compressedSize[i], U = uncompressedSize[i];
        hb[k] = io; hb[m + k] = C; hb[2 * m + k] = oo; hb[3 * m + k] = U;
        memcpy(c->h_in + io, data[i], C);
        io += round16(C);
        oo += round16(U);
    }
    const uint64_t t1 = now_ns();
    uint64_t* db = reinterpret_cast<uint64_t*>(c->d_bm);
    uint32_t* d_status = reinterpret_cast<uint32_t*>(db + 4 * m);
    check(hipMemcpyAsync(c->d_in, c->h_in, inTot, hipMemcpyHostToDevice, c->s), "H2D");
    check(hipMemcpyAsync(db, hb, 32 * m, hipMemcpyHostToDevice, c->s), "H2D(meta)");
    if (mL && rle_decode_batch_device_seg(c->d_in, db, db + m, c->d_out, db + 2 * m, db + 3 * m, nullptr, d_status,
                                          (uint32_t)mL, inLarge, c->d_ws, c->d_ws_cap, c->s) != RLE_OK)
        die("decode launch", hipGetLastError());
    if (m > mL && rle_decode_batch_device_sized(c->d_in, db + mL, db + m + mL, c->d_out, db + 2 * m + mL, db + 3 * m + mL,
                                                nullptr, d_status + mL, (uint32_t)(m - mL), maxCs, maxUs, c->s) != RLE_OK)
        die("decode launch", hipGetLastError());
    check(hipMemcpyAsync(c->h_out, c->d_out, outTot, hipMemcpyDeviceToHost, c->s), "D2H");
    check(hipMemcpyAsync(hb + 4 * m, d_status, 4 * m, hipMemcpyDeviceToHost, c->s), "D2H(status)");
    check(hipStreamSynchronize(c->s), "hipStreamSynchronize");
    const uint64_t t2 = now_ns();
    const uint32_t* hst = reinterpret_cast<const uint32_t*>(hb + 4 * m);
    for (size_t k = 0; k < m; ++k) {
        const size_t i = idx[k], U = uncompressedSize[i];
        if (U) memcpy(out[i], c->h_out + hb[2 * m + k], U);
        if (hst[k] & RLE_STATUS_OVERFLOW) warn_overflow("RLEdecompressN");
    }
    t.ns_in += t1 - t0;
    t.ns_dev += t2 - t1;
    t.ns_out += now_ns() - t2;
    t.h2d += inTot;
    t.d2h += outTot;
}

// A chunk of small files through this thread's mapped buffer (round 6; g_zerocopy): the streams
// copied into its input region, one launch over them, the decoded files written into its output
// region, the per-file status words polled (each stored behind a system-scope release of its file),
// no copy commands.  Files a one-wave or cooperative decode takes (zc_n_fits), at most kZcNFiles
// (the metadata fits the words region) and the mapped regions' bytes per chunk.
// (Files up to 16 KiB: a 64 KiB file's one-wave decode writing over PCIe took 200 µs per chunk of
// five, r6aa: 64 x 64 KiB zero 2266 µs against 456 staged.)
constexpr size_t kZcNFiles = 56;   // 36 bytes of launch words each, below kZcWords + 2048 (kZcMail)
constexpr size_t kZcNMaxU = 16384;
bool zc_n_fits(size_t C, size_t U) {
    return g_zerocopy && C < kSegDecodeBytes && U <= kZcNMaxU;
}
void decompress_n_chunk_zc(Ctx* c, const size_t* idx, size_t m, char* const* data, const size_t* compressedSize,
                           const size_t* uncompressedSize, char* const* out, NTotals& t) {
    uint8_t* h = zc(c);
    uint64_t* hw = reinterpret_cast<uint64_t*>(h + kZcWords);
    uint64_t* dw = reinterpret_cast<uint64_t*>(c->d_zc + kZcWords);
    uint32_t* hst = reinterpret_cast<uint32_t*>(hw + 4 * m);
    const uint64_t t0 = now_ns();
    size_t io = 0, oo = 0, maxC = 0, maxU = 0;
    for (size_t k = 0; k < m; ++k) {
        const size_t i = idx[k], C = compressedSize[i], U = uncompressedSize[i];
        hw[k] = kZcIn + io; hw[m + k] = C; hw[2 * m + k] = kZcOut + oo; hw[3 * m + k] = U;
        hst[k] = kPending;
        memcpy(h + kZcIn + io, data[i], C);
        io += round16(C);
        oo += round16(U);
        maxC = std::max(maxC, C);
        maxU = std::max(maxU, U);
    }
    const uint64_t t1 = now_ns();
    if (rle_decode_batch_device_sized_flags(c->d_zc, dw, dw + m, c->d_zc, dw + 2 * m, dw + 3 * m, nullptr,
                                            reinterpret_cast<uint32_t*>(dw + 4 * m), (uint32_t)m, maxC, maxU,
                                            RLE_LAUNCH_STATUS_FLAG, c->s) != RLE_OK)
        die("decode launch", hipGetLastError());
    // every file's status (the launch's last stores are in no particular order); zc_wait's bounds
    // and periodic synchronize, counted once per launch
    const uint32_t polled = c->polled;
    for (size_t k = 0; k < m; ++k) {
        c->polled = polled;
        (void)zc_wait(c, reinterpret_cast<const uint64_t*>(hst + k));
    }
    const uint64_t t2 = now_ns();
    for (size_t k = 0; k < m; ++k) {
        const size_t i = idx[k], U = uncompressedSize[i];
        if (U) memcpy(out[i], h + hw[2 * m + k], U);
        if (hst[k] & RLE_STATUS_OVERFLOW) warn_overflow("RLEdecompressN");
    }
    t.ns_in += t1 - t0;
    t.ns_dev += t2 - t1;
    t.ns_out += now_ns() - t2;
    t.h2d += io;
    t.d2h += oo;
}

int decompress_n_impl(size_t n, char* const* data, const size_t* compressedSize, const size_t* uncompressedSize,
                      char* const* out) {
    std::vector<size_t> idx;
    idx.reserve(n);
    for (size_t i = 0; i < n; ++i) {
        const size_t C = compressedSize[i], U = uncompressedSize[i];
        if (C == 0) {  // calloc'd block (src/rleCompression.c:48)
            if (U) memset(out[i], 0, U);
            continue;
        }
        if (!data[i] || (U && !out[i])) {
            errno = EINVAL;
            return -1;
        }
        if (too_big("RLEdecompressN", C) || too_big("RLEdecompressN", U)) return -1;
        idx.push_back(i);
    }
    if (idx.empty()) return 0;
    Ctx* c = ctx();
    NTotals t;
    // files in batch order: chunks of consecutive small files through the mapped buffer (zc_n_fits),
    // chunks of consecutive files that fit the staging together, files too large for it alone
    size_t k0 = 0, inTot = 0, outTot = 0;
    bool zcChunk = false;
    for (size_t k = 0; k <= idx.size(); ++k) {
        const bool end = k == idx.size();
        const size_t Ci = end ? 0 : round16(compressedSize[idx[k]]), Ui = end ? 0 : round16(uncompressedSize[idx[k]]);
        const bool zcFile = !end && zc_n_fits(compressedSize[idx[k]], uncompressedSize[idx[k]]);
        const bool alone = !end && (Ci > g_stage_cap || Ui > g_stage_cap);
        const bool full = zcChunk ? (inTot + Ci > kZcWords || outTot + Ui > kZcMaxOut || k - k0 >= kZcNFiles)
                                  : (inTot + Ci > g_stage_cap || outTot + Ui > g_stage_cap);
        if (end || alone || full || (k > k0 && zcFile != zcChunk)) {
            if (k > k0 && zcChunk)
                decompress_n_chunk_zc(c, idx.data() + k0, k - k0, data, compressedSize, uncompressedSize, out, t);
            else if (k > k0)
                decompress_n_chunk(c, idx.data() + k0, k - k0, data, compressedSize, uncompressedSize, out, t);
            k0 = k;
            inTot = outTot = 0;
        }
        zcChunk = zcFile;
        if (alone) {
            const size_t i = idx[k];
            decompress_n_alone(c, data[i], compressedSize[i], uncompressedSize[i], out[i], t);
            k0 = k + 1;
            continue;
        }
        inTot += Ci;
        outTot += Ui;
    }
    for (size_t i : idx) {
        t.cin += compressedSize[i];
        t.uout += uncompressedSize[i];
    }
    g_stats.calls_decompress += idx.size();
    g_stats.bytes_in += t.cin;
    g_stats.bytes_out += t.uout;
    g_stats.bytes_h2d += t.h2d;
    g_stats.bytes_d2h += t.d2h;
    g_stats.ns_stage_in += t.ns_in;
    g_stats.ns_device += t.ns_dev;
    g_stats.ns_stage_out += t.ns_out;
    return 0;
}
}  // namespace

// readNFilesHandler's decode loop (src/filesystemApi.c:675-687) and the
// eviction loop (src/server.c:314-323) as batched launches (include/rle_fileops.h).  Files are
// staged in bounded chunks (g_stage_cap), so the pinned memory a worker thread holds does not grow
// with the batch.
extern "C" int RLEdecompressN(size_t n, char* const* data, const size_t* compressedSize,
                              const size_t* uncompressedSize, char* const* out) {
    TraceScope ts('n', n, 0, 0);
    if (n == 0) return 0;
    if (!data || !compressedSize || !uncompressedSize || !out) {
        errno = EINVAL;
        return -1;
    }
    try {
        return decompress_n_impl(n, data, compressedSize, uncompressedSize, out);
    } catch (const std::bad_alloc&) {
        drain_after_oom();
        return -1;
    }
}

extern "C" int rle_mi355x_dropin_stats(rle_dropin_stats_t* out, int reset) {
    if (!out) return RLE_E_INVAL;
    out->calls_compress = g_stats.calls_compress.load();
    out->calls_decompress = g_stats.calls_decompress.load();
    out->calls_append = g_stats.calls_append.load();
    out->bytes_in = g_stats.bytes_in.load();
    out->bytes_out = g_stats.bytes_out.load();
    out->bytes_h2d = g_stats.bytes_h2d.load();
    out->bytes_d2h = g_stats.bytes_d2h.load();
    out->ns_stage_in = g_stats.ns_stage_in.load();
    out->ns_device = g_stats.ns_device.load();
    out->ns_stage_out = g_stats.ns_stage_out.load();
    out->calls_coalesced = g_stats.calls_coalesced.load();
    out->launches_coalesced = g_stats.launches_coalesced.load();
    out->calls_registered = g_stats.calls_registered.load();
    out->calls_reg_fallback = g_stats.calls_reg_fallback.load();
    if (reset) {
        g_stats.calls_compress = 0; g_stats.calls_decompress = 0; g_stats.calls_append = 0; g_stats.bytes_in = 0; g_stats.bytes_out = 0;
        g_stats.bytes_h2d = 0; g_stats.bytes_d2h = 0; g_stats.ns_stage_in = 0; g_stats.ns_device = 0;
        g_stats.ns_stage_out = 0;
        g_stats.calls_coalesced = 0;
        g_stats.launches_coalesced = 0;
        g_stats.calls_registered = 0;
        g_stats.calls_reg_fallback = 0;
    }
    return RLE_OK;
}

namespace {
// RLE_MI355X_STATS=<path>: the drop-in's host-path accounting is written there as JSON at exit
// (used to record the server's host<->device rate).
struct StatsAtExit {
    ~StatsAtExit() {
        if (g_trace) {
            if (FILE* f = fopen(getenv("RLE_MI355X_TRACE"), "w")) {
                const uint32_t n = std::min(g_trace_n.load(), kTraceMax);
                for (uint32_t i = 0; i < n; ++i) {
                    const TraceRec& t = g_trace[i];
                    fprintf(f, "%c %u %llu %llu %llu %llu %llu %llu\n", t.op, t.tid, (unsigned long long)t.a,
                            (unsigned long long)t.b, (unsigned long long)t.c, (unsigned long long)t.t0,
                            (unsigned long long)t.dt, (unsigned long long)t.ctx_ns);
                }
                fclose(f);
            }
        }
        const char* path = getenv("RLE_MI355X_STATS");
        if (!path || !*path) return;
        rle_dropin_stats_t s;
        rle_mi355x_dropin_stats(&s, 0);
        FILE* f = fopen(path, "w");
        if (!f) return;
        fprintf(f,
                "{\"calls_compress\": %llu, \"calls_decompress\": %llu, \"calls_append\": %llu, \"bytes_in\": %llu, \"bytes_out\": %llu, "
                "\"bytes_h2d\": %llu, \"bytes_d2h\": %llu, \"ns_stage_in\": %llu, \"ns_device\": %llu, "
                "\"ns_stage_out\": %llu, \"calls_coalesced\": %llu, \"launches_coalesced\": %llu}\n",
                (unsigned long long)s.calls_compress, (unsigned long long)s.calls_decompress,
                (unsigned long long)s.calls_append,
                (unsigned long long)s.bytes_in, (unsigned long long)s.bytes_out, (unsigned long long)s.bytes_h2d,
                (unsigned long long)s.bytes_d2h, (unsigned long long)s.ns_stage_in, (unsigned long long)s.ns_device,
                (unsigned long long)s.ns_stage_out, (unsigned long long)s.calls_coalesced,
                (unsigned long long)s.launches_coalesced);
        fclose(f);
    }
} g_stats_at_exit;
}  // namespace
