// rle_dropin.cpp — the drop-in C ABI of include/rleCompression.h on top of the MI355X kernels.
//
// Replaces src/rleCompression.c:9-62 (samul-1/C-FileStorage-Server-and-Client) for its callers
// src/filesystemApi.c:597 (read), :680 (readNFiles), :767/:774 (write/append = decode, append,
// re-encode) and src/server.c:317 (evicted files), which link against this library unchanged.
//
// Each calling thread (the server's worker pool, src/server.c:520-524) gets its own HIP stream,
// pinned host staging and device buffers, created lazily on its first call (there is no init
// hook in the server, src/server.c:406-524) and released at thread exit.  A call is: copy the
// caller's bytes into pinned staging -> H2D -> one batched kernel launch with B = 1 -> D2H ->
// copy into a fresh malloc() block, which is what the callers free() (src/filesystemApi.c:208,
// 687, 775, 811; src/server.c:269, 320).  There is no CPU codec in this library: without a
// usable GPU it reports the problem and aborts.
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>

#include "rleCompression.h"
#include "rle_mi355x.h"

namespace {

pthread_once_t g_once = PTHREAD_ONCE_INIT;
pthread_key_t g_key;
int g_ndev = 0;
int g_dev_pin = -1;
std::atomic<unsigned> g_next_dev{0};
std::atomic<int> g_warned_overflow{0};

// Host-path accounting (rle_mi355x_dropin_stats): bytes moved and wall time per phase.
struct Stats {
    std::atomic<uint64_t> calls_compress{0}, calls_decompress{0};
    std::atomic<uint64_t> bytes_in{0}, bytes_out{0};        // caller bytes in / returned bytes out
    std::atomic<uint64_t> bytes_h2d{0}, bytes_d2h{0};
    std::atomic<uint64_t> ns_stage_in{0}, ns_device{0}, ns_stage_out{0};
} g_stats;
inline uint64_t now_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}

[[noreturn]] void die(const char* what, hipError_t e) {
    fprintf(stderr, "librle_mi355x: %s failed: %s\n", what, hipGetErrorString(e));
    abort();
}
inline void check(hipError_t e, const char* what) {
    if (e != hipSuccess) die(what, e);
}

// Small-call threshold: up to this many input bytes the worst-case output is copied back in the
// same round trip as its size (one stream sync instead of two).
constexpr size_t kOneTripBytes = 128u << 10;
// From these sizes one call is cut into segments processed by separate waves
// (rle_*_batch_device_seg) instead of one wave walking the whole buffer.
constexpr size_t kSegEncodeBytes = 48u << 10;
constexpr size_t kSegDecodeBytes = 32u << 10;

struct Ctx {
    int dev = 0;
    hipStream_t s = nullptr;
    uint8_t* h_in = nullptr;  size_t h_in_cap = 0;    // pinned staging: caller bytes -> device
    uint8_t* h_out = nullptr; size_t h_out_cap = 0;   // pinned staging: device -> caller block
    uint8_t* d_in = nullptr;  size_t d_in_cap = 0;
    uint8_t* d_out = nullptr; size_t d_out_cap = 0;
    uint64_t* d_meta = nullptr;                      // [in_off, in_len, out_off, out_len, out_cap, status]
    uint64_t* h_meta = nullptr;                      // pinned mirror
    uint8_t* d_ws = nullptr;  size_t d_ws_cap = 0;    // segmented-path workspace
};

// A worker thread's context is released by its pthread-key destructor, which can still be running
// when the process exits (a thread joined by its creator has not necessarily finished its TLS
// destructors).  Process exit tears the HIP runtime down, so from the first atexit handler on no
// context touches HIP any more (the OS reclaims the memory); the lock orders the two.
pthread_mutex_t g_exit_lock = PTHREAD_MUTEX_INITIALIZER;
bool g_exiting = false;
void on_exit_handler() {
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
    (void)hipSetDevice(c->dev);
    if (c->s) (void)hipStreamSynchronize(c->s);
    (void)hipHostFree(c->h_in);
    (void)hipHostFree(c->h_out);
    (void)hipHostFree(c->h_meta);
    (void)hipFree(c->d_in);
    (void)hipFree(c->d_out);
    (void)hipFree(c->d_meta);
    (void)hipFree(c->d_ws);
    if (c->s) (void)hipStreamDestroy(c->s);
    delete c;
    pthread_mutex_unlock(&g_exit_lock);
}

void init_once() {
    if (hipGetDeviceCount(&g_ndev) != hipSuccess) g_ndev = 0;
    if (const char* e = getenv("RLE_MI355X_DEVICE")) g_dev_pin = atoi(e);
    pthread_key_create(&g_key, free_ctx);
    atexit(on_exit_handler);   // registered after the HIP runtime's own exit hooks: runs before them
}

inline size_t round16(size_t x) { return (x + 15u) & ~(size_t)15u; }

Ctx* ctx() {
    pthread_once(&g_once, init_once);
    Ctx* c = static_cast<Ctx*>(pthread_getspecific(g_key));
    if (c) {
        check(hipSetDevice(c->dev), "hipSetDevice");
        return c;
    }
    if (g_ndev <= 0) {
        fprintf(stderr, "librle_mi355x: no HIP device is visible; the RLE codec runs on MI355X only\n");
        abort();
    }
    c = new Ctx();
    c->dev = (g_dev_pin >= 0 && g_dev_pin < g_ndev) ? g_dev_pin : (int)(g_next_dev++ % (unsigned)g_ndev);
    check(hipSetDevice(c->dev), "hipSetDevice");
    check(hipStreamCreateWithFlags(&c->s, hipStreamNonBlocking), "hipStreamCreate");
    check(hipMalloc(&c->d_meta, 8 * sizeof(uint64_t)), "hipMalloc(meta)");
    check(hipHostMalloc(&c->h_meta, 8 * sizeof(uint64_t), hipHostMallocDefault), "hipHostMalloc(meta)");
    pthread_setspecific(g_key, c);
    return c;
}

void grow_host(uint8_t*& p, size_t& cap, size_t need) {
    if (need <= cap) return;
    size_t n = cap ? cap : (64u << 10);
    while (n < need) n *= 2;
    if (p) check(hipHostFree(p), "hipHostFree");
    check(hipHostMalloc(reinterpret_cast<void**>(&p), n, hipHostMallocDefault), "hipHostMalloc");
    cap = n;
}
void grow_dev(uint8_t*& p, size_t& cap, size_t need) {
    if (need <= cap) return;
    size_t n = cap ? cap : (64u << 10);
    while (n < need) n *= 2;
    if (p) check(hipFree(p), "hipFree");
    check(hipMalloc(reinterpret_cast<void**>(&p), n), "hipMalloc");
    cap = n;
}

}  // namespace

// src/rleCompression.c:9-45 — returns a malloc block: C token bytes + >= 2 zero bytes.
extern "C" char* RLEcompress(char* data, size_t origSize, size_t* compressedSize) {
    const size_t U = origSize;
    if (U == 0) {
        *compressedSize = 0;
        return static_cast<char*>(calloc(16, 1));
    }
    Ctx* c = ctx();
    const size_t maxC = rle_max_compressed_size(U);
    grow_host(c->h_in, c->h_in_cap, U);
    grow_dev(c->d_in, c->d_in_cap, round16(U));
    grow_dev(c->d_out, c->d_out_cap, round16(maxC));
    const uint64_t t0 = now_ns();
    memcpy(c->h_in, data, U);
    const uint64_t t1 = now_ns();
    c->h_meta[0] = 0; c->h_meta[1] = U; c->h_meta[2] = 0; c->h_meta[3] = 0;
    check(hipMemcpyAsync(c->d_in, c->h_in, U, hipMemcpyHostToDevice, c->s), "H2D");
    check(hipMemcpyAsync(c->d_meta, c->h_meta, 4 * sizeof(uint64_t), hipMemcpyHostToDevice, c->s), "H2D(meta)");
    uint32_t* d_status = reinterpret_cast<uint32_t*>(c->d_meta + 5);
    if (U >= kSegEncodeBytes) grow_dev(c->d_ws, c->d_ws_cap, rle_seg_workspace_bytes(1, U));
    const int erc = U >= kSegEncodeBytes
                        ? rle_encode_batch_device_seg(c->d_in, c->d_meta + 0, c->d_meta + 1, c->d_out, c->d_meta + 2,
                                                      c->d_meta + 3, d_status, 1, U, c->d_ws, c->d_ws_cap, c->s)
                        : rle_encode_batch_device(c->d_in, c->d_meta + 0, c->d_meta + 1, c->d_out, c->d_meta + 2,
                                                  c->d_meta + 3, d_status, 1, c->s);
    if (erc != RLE_OK) die("encode launch", hipGetLastError());
    check(hipMemcpyAsync(c->h_meta + 3, c->d_meta + 3, sizeof(uint64_t), hipMemcpyDeviceToHost, c->s), "D2H(meta)");
    const bool one_trip = U <= kOneTripBytes;
    if (one_trip) {
        grow_host(c->h_out, c->h_out_cap, maxC);
        check(hipMemcpyAsync(c->h_out, c->d_out, maxC, hipMemcpyDeviceToHost, c->s), "D2H");
    }
    check(hipStreamSynchronize(c->s), "hipStreamSynchronize");
    const size_t C = c->h_meta[3];
    if (!one_trip) {
        grow_host(c->h_out, c->h_out_cap, C);
        check(hipMemcpyAsync(c->h_out, c->d_out, C, hipMemcpyDeviceToHost, c->s), "D2H");
        check(hipStreamSynchronize(c->s), "hipStreamSynchronize");
    }
    const uint64_t t2 = now_ns();
    char* r = static_cast<char*>(malloc(C + 16));
    if (!r) {
        *compressedSize = C;
        return nullptr;
    }
    memcpy(r, c->h_out, C);
    memset(r + C, 0, 16);
    *compressedSize = C;
    const uint64_t t3 = now_ns();
    g_stats.calls_compress++;
    g_stats.bytes_in += U;
    g_stats.bytes_out += C;
    g_stats.bytes_h2d += U;
    g_stats.bytes_d2h += one_trip ? maxC : C;
    g_stats.ns_stage_in += t1 - t0;
    g_stats.ns_device += t2 - t1;
    g_stats.ns_stage_out += t3 - t2;
    return r;
}

// src/rleCompression.c:47-62 — returns a malloc block of U+E bytes (decoded U, then E zeros).
extern "C" char* RLEdecompress(char* data, size_t compressedSize, size_t uncompressedSize, size_t extraAllocation) {
    const size_t C = compressedSize, U = uncompressedSize, E = extraAllocation, total = U + E;
    char* r = static_cast<char*>(malloc(total ? total : 1));
    if (!r) return nullptr;
    if (C == 0) {  // nothing to decode: calloc'd block (:48)
        memset(r, 0, total);
        return r;
    }
    Ctx* c = ctx();
    grow_host(c->h_in, c->h_in_cap, C);
    grow_host(c->h_out, c->h_out_cap, total);
    grow_dev(c->d_in, c->d_in_cap, round16(C));
    grow_dev(c->d_out, c->d_out_cap, round16(total));
    const uint64_t t0 = now_ns();
    memcpy(c->h_in, data, C);
    const uint64_t t1 = now_ns();
    c->h_meta[0] = 0; c->h_meta[1] = C; c->h_meta[2] = 0; c->h_meta[3] = U; c->h_meta[4] = total; c->h_meta[5] = 0;
    check(hipMemcpyAsync(c->d_in, c->h_in, C, hipMemcpyHostToDevice, c->s), "H2D");
    check(hipMemcpyAsync(c->d_meta, c->h_meta, 6 * sizeof(uint64_t), hipMemcpyHostToDevice, c->s), "H2D(meta)");
    uint32_t* d_status = reinterpret_cast<uint32_t*>(c->d_meta + 5);
    if (C >= kSegDecodeBytes) grow_dev(c->d_ws, c->d_ws_cap, rle_seg_workspace_bytes(1, C));
    const int drc = C >= kSegDecodeBytes
                        ? rle_decode_batch_device_seg(c->d_in, c->d_meta + 0, c->d_meta + 1, c->d_out, c->d_meta + 2,
                                                      c->d_meta + 3, c->d_meta + 4, d_status, 1, C, c->d_ws,
                                                      c->d_ws_cap, c->s)
                        : rle_decode_batch_device(c->d_in, c->d_meta + 0, c->d_meta + 1, c->d_out, c->d_meta + 2,
                                                  c->d_meta + 3, c->d_meta + 4, d_status, 1, c->s);
    if (drc != RLE_OK) die("decode launch", hipGetLastError());
    check(hipMemcpyAsync(c->h_meta + 5, c->d_meta + 5, sizeof(uint64_t), hipMemcpyDeviceToHost, c->s), "D2H(meta)");
    if (U) check(hipMemcpyAsync(c->h_out, c->d_out, U, hipMemcpyDeviceToHost, c->s), "D2H");
    check(hipStreamSynchronize(c->s), "hipStreamSynchronize");
    const uint32_t st = (uint32_t)c->h_meta[5];
    const uint64_t t2 = now_ns();
    memcpy(r, c->h_out, U);
    if (E) {
        if (st & RLE_STATUS_SERIAL) {  // a non-encoder stream may have written into the E region
            check(hipMemcpyAsync(c->h_out + U, c->d_out + U, E, hipMemcpyDeviceToHost, c->s), "D2H");
            check(hipStreamSynchronize(c->s), "hipStreamSynchronize");
            memcpy(r + U, c->h_out + U, E);
        } else {
            memset(r + U, 0, E);
        }
    }
    if ((st & RLE_STATUS_OVERFLOW) && !g_warned_overflow.exchange(1))
        fprintf(stderr, "librle_mi355x: RLEdecompress: stream decodes past U+E (the reference would overflow its "
                        "heap block); output truncated\n");
    const uint64_t t3 = now_ns();
    g_stats.calls_decompress++;
    g_stats.bytes_in += C;
    g_stats.bytes_out += total;
    g_stats.bytes_h2d += C;
    g_stats.bytes_d2h += U;
    g_stats.ns_stage_in += t1 - t0;
    g_stats.ns_device += t2 - t1;
    g_stats.ns_stage_out += t3 - t2;
    return r;
}

extern "C" int rle_mi355x_dropin_stats(rle_dropin_stats_t* out, int reset) {
    if (!out) return RLE_E_INVAL;
    out->calls_compress = g_stats.calls_compress.load();
    out->calls_decompress = g_stats.calls_decompress.load();
    out->bytes_in = g_stats.bytes_in.load();
    out->bytes_out = g_stats.bytes_out.load();
    out->bytes_h2d = g_stats.bytes_h2d.load();
    out->bytes_d2h = g_stats.bytes_d2h.load();
    out->ns_stage_in = g_stats.ns_stage_in.load();
    out->ns_device = g_stats.ns_device.load();
    out->ns_stage_out = g_stats.ns_stage_out.load();
    if (reset) {
        g_stats.calls_compress = 0; g_stats.calls_decompress = 0; g_stats.bytes_in = 0; g_stats.bytes_out = 0;
        g_stats.bytes_h2d = 0; g_stats.bytes_d2h = 0; g_stats.ns_stage_in = 0; g_stats.ns_device = 0;
        g_stats.ns_stage_out = 0;
    }
    return RLE_OK;
}

namespace {
// RLE_MI355X_STATS=<path>: the drop-in's host-path accounting is written there as JSON at exit
// (used to record the server's host<->device rate).
struct StatsAtExit {
    ~StatsAtExit() {
        const char* path = getenv("RLE_MI355X_STATS");
        if (!path || !*path) return;
        rle_dropin_stats_t s;
        rle_mi355x_dropin_stats(&s, 0);
        FILE* f = fopen(path, "w");
        if (!f) return;
        fprintf(f,
                "{\"calls_compress\": %llu, \"calls_decompress\": %llu, \"bytes_in\": %llu, \"bytes_out\": %llu, "
                "\"bytes_h2d\": %llu, \"bytes_d2h\": %llu, \"ns_stage_in\": %llu, \"ns_device\": %llu, "
                "\"ns_stage_out\": %llu}\n",
                (unsigned long long)s.calls_compress, (unsigned long long)s.calls_decompress,
                (unsigned long long)s.bytes_in, (unsigned long long)s.bytes_out, (unsigned long long)s.bytes_h2d,
                (unsigned long long)s.bytes_d2h, (unsigned long long)s.ns_stage_in, (unsigned long long)s.ns_device,
                (unsigned long long)s.ns_stage_out);
        fclose(f);
    }
} g_stats_at_exit;
}  // namespace
