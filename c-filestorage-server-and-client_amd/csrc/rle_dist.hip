// rle_dist.hip — the multi-GPU exchange step of bench.py / shard.py at N > 1:
// each rank's per-buffer compressed sizes all-gathered over RCCL (xGMI) and scanned into offsets
// in the global stream order (buffer i = k * world + r is rank r's k-th buffer).
//
// A step's exchange is one C call on the host (rle_dist_gather_offsets): ncclAllGather straight
// from the sizes and the reorder + exclusive scan kernel, on the caller's stream between its encode
// and its decode.  Issued from Python as separate torch calls on a side stream the same exchange
// cost 56-87 us of host time per configs[1] step against ~21 us of GPU time; this call costs
// ~7 us (tools/exchange_cost.py: 17.5 us enqueue, 28 us wall per step with one rank).  A side
// stream measured worse: its event handshakes cost more host and GPU time than the overlap saved
// (36.6 us enqueue, 45 us wall).
//
// RCCL is resolved at run time (dlopen / dlsym) from the copy the process already loaded (torch's
// librccl.so.1) or from an explicit path: the codec library links no second RCCL.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "rle_mi355x.h"

namespace {

typedef int ncclResult_t;   // ncclSuccess == 0
typedef struct ncclComm* ncclComm_t;
struct ncclUniqueId {
    char internal[128];   // NCCL_UNIQUE_ID_BYTES
};
constexpr int kNcclInt64 = 4;   // ncclDataType_t ncclInt64 (rccl.h)

struct Rccl {
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*all_gather)(const void*, void*, size_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    bool ok = false;
};

Rccl g_rccl;
ncclComm_t g_comm = nullptr;
int g_world = 0;
bool load_rccl(const char* path) {
    if (g_rccl.ok) return true;
    void* h = nullptr;
    if (path && *path) h = dlopen(path, RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);
    if (!h) return false;
    g_rccl.get_unique_id = (decltype(g_rccl.get_unique_id))dlsym(h, "ncclGetUniqueId");
    g_rccl.comm_init_rank = (decltype(g_rccl.comm_init_rank))dlsym(h, "ncclCommInitRank");
    g_rccl.all_gather = (decltype(g_rccl.all_gather))dlsym(h, "ncclAllGather");
    g_rccl.comm_destroy = (decltype(g_rccl.comm_destroy))dlsym(h, "ncclCommDestroy");
    g_rccl.ok = g_rccl.get_unique_id && g_rccl.comm_init_rank && g_rccl.all_gather && g_rccl.comm_destroy;
    return g_rccl.ok;
}

// The reorder + exclusive scan, over the whole chip (until r3 one workgroup walked all entries on
// one CU).  gathered is rank major -- global buffer i = k * world + r sits at gathered[r * n + k].
// A sub-tile is T consecutive k of every rank: each rank's part is one contiguous, coalesced run,
// and its world * T outputs are one contiguous run of the global order.  A workgroup takes `items`
// consecutive sub-tiles, so that there are at most kMaxTiles workgroups.
//   tile_sums_kernel   each workgroup sums its sub-tiles into ws[t];
//   tile_scan_kernel   each workgroup adds up ws[0, t), then per sub-tile: thread j loads k = kb + j
//                      of every rank into registers (world W a template constant up to 16), a
//                      workgroup scan gives each k's offset, the W offsets of k go to LDS in global
//                      order and leave as one coalesced run.
// Exchanges of at most kSmallK sizes per rank take one launch: a single 512-thread workgroup, one
// sub-tile, no workspace.  (A single workgroup walking several sub-tiles in turn is slower than the
// two launches: 17.4 us for 8 x 4096 against ~3-6 us per kernel, r3d rocprof.)  At 1 M entries the
// two kernels take 10-12 us together (8 x 131072, r3d).  No division anywhere.
constexpr unsigned kScanThreads = 256, kSmallThreads = 512, kMaxTiles = 2048;
constexpr size_t kStageBytes = 32768;   // LDS staging of one sub-tile's outputs, at most
constexpr uint32_t kSmallK = kSmallThreads;

template <unsigned T>
__device__ __forceinline__ int64_t block_sum(int64_t v, int64_t* red) {
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    __syncthreads();   // red may still be read from a previous call
    if ((threadIdx.x & 63u) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    int64_t s = 0;
    for (unsigned k = 0; k < T / 64; ++k) s += red[k];
    return s;
}

// exclusive scan over the workgroup; *total = the workgroup's sum
template <unsigned T>
__device__ __forceinline__ int64_t block_excl_scan(int64_t v, int64_t* red, int64_t* total) {
    const unsigned lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    int64_t x = v;
    for (unsigned d = 1; d < 64u; d <<= 1) {
        const int64_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    __syncthreads();
    if (lane == 63u) red[w] = x;
    __syncthreads();
    int64_t before = 0, all = 0;
    for (unsigned k = 0; k < T / 64; ++k) {
        if (k < w) before += red[k];
        all += red[k];
    }
    *total = all;
    return before + x - v;
}

__global__ __launch_bounds__(kScanThreads) void tile_sums_kernel(const int64_t* __restrict__ gathered, uint32_t world,
                                                                 uint32_t n, uint32_t items, int64_t* __restrict__ ws) {
    __shared__ int64_t red[kScanThreads / 64];
    const uint64_t k0 = (uint64_t)blockIdx.x * items * kScanThreads;
    const uint64_t k1 = k0 + (uint64_t)items * kScanThreads < n ? k0 + (uint64_t)items * kScanThreads : n;
    int64_t s = 0;
    for (uint32_t r = 0; r < world; ++r) {
        const int64_t* g = gathered + (uint64_t)r * n;
        for (uint64_t k = k0 + threadIdx.x; k < k1; k += kScanThreads) s += g[k];   // coalesced
    }
    s = block_sum<kScanThreads>(s, red);
    if (threadIdx.x == 0) ws[blockIdx.x] = s;
}

// W: the world size (1..16) as a constant, or 0 (any world: direct stores, no staging).  ws == NULL:
// a single workgroup (the prefix before it is 0).
template <unsigned W, unsigned T>
__global__ __launch_bounds__(T) void tile_scan_kernel(const int64_t* __restrict__ gathered, uint32_t world, uint32_t n,
                                                      uint32_t items, const int64_t* __restrict__ ws,
                                                      int64_t* __restrict__ out) {
    __shared__ int64_t red[T / 64];
    __shared__ int64_t stage[W ? W * T : 1];
    constexpr unsigned WR = W ? W : 1;
    int64_t carry = 0;   // the sum of every workgroup's part before this one
    {
        int64_t pre = 0;
        if (ws)
            for (uint32_t t = threadIdx.x; t < blockIdx.x; t += T) pre += ws[t];
        carry = block_sum<T>(pre, red);
    }
    for (uint32_t sub = 0; sub < items; ++sub) {
        const uint64_t kb = ((uint64_t)blockIdx.x * items + sub) * T;
        if (kb >= n) break;
        const uint64_t k = kb + threadIdx.x;
        const bool valid = k < n;
        int64_t v[WR];
        int64_t mine = 0;
        if (W) {
#pragma unroll
            for (unsigned r = 0; r < WR; ++r) {
                v[r] = valid ? gathered[(uint64_t)r * n + k] : 0;
                mine += v[r];
            }
        } else if (valid) {
            for (uint32_t r = 0; r < world; ++r) mine += gathered[(uint64_t)r * n + k];
        }
        int64_t total;
        int64_t run = carry + block_excl_scan<T>(mine, red, &total);
        if (W) {
#pragma unroll
            for (unsigned r = 0; r < WR; ++r) {
                stage[threadIdx.x * WR + r] = run;
                run += v[r];
            }
            __syncthreads();
            const uint64_t cnt = (n - kb < T ? n - kb : T) * (uint64_t)WR;
            int64_t* o = out + kb * WR;
            for (uint64_t j = threadIdx.x; j < cnt; j += T) o[j] = stage[j];   // coalesced
        } else if (valid) {
            for (uint32_t r = 0; r < world; ++r) {
                out[k * world + r] = run;
                run += gathered[(uint64_t)r * n + k];
            }
        }
        carry += total;
    }
}

template <unsigned T>
void launch_scan(uint32_t grid, hipStream_t s, const int64_t* g, uint32_t world, uint32_t n, uint32_t items,
                 const int64_t* ws, int64_t* out) {
#define RLE_SCAN(W) hipLaunchKernelGGL((tile_scan_kernel<(W * T * 8u <= kStageBytes ? W : 0u), T>), dim3(grid), dim3(T), \
                                       0, s, g, world, n, items, ws, out)
    switch (world) {
        case 1: RLE_SCAN(1); break;
        case 2: RLE_SCAN(2); break;
        case 3: RLE_SCAN(3); break;
        case 4: RLE_SCAN(4); break;
        case 8: RLE_SCAN(8); break;
        case 16: RLE_SCAN(16); break;
        default: RLE_SCAN(0); break;
    }
#undef RLE_SCAN
}

// Tile sums of the whole-chip scan: tiles(n) int64 in the CALLER's workspace (round 4: a process-wide
// workspace per device was shared by every caller, so two scans with n > kSmallK queued on different
// streams of one device could write each other's tile sums, and a grown workspace was freed under a
// HIP graph that had captured the old pointer).  Each caller now passes its own: exchanges that may
// run at once (the two slots of shard.NativeExchange) use different workspaces, and a captured graph
// keeps pointing at memory its owner keeps alive.
uint32_t scan_tiles(uint32_t n, uint32_t* items_out) {
    const uint32_t subtiles = (uint32_t)(((uint64_t)n + kScanThreads - 1) / kScanThreads);
    const uint32_t items = (subtiles + kMaxTiles - 1) / kMaxTiles;
    if (items_out) *items_out = items;
    return (subtiles + items - 1) / items;
}

}  // namespace

extern "C" size_t rle_dist_workspace_bytes(uint32_t n) {
    return n <= kSmallK ? 0u : (size_t)scan_tiles(n, nullptr) * sizeof(int64_t);
}

extern "C" int rle_dist_offsets_device(const int64_t* d_gathered, uint32_t world, uint32_t n, int64_t* d_offsets,
                                       void* d_ws, size_t ws_bytes, void* stream) {
    if (!d_gathered || !d_offsets || world == 0) return RLE_E_INVAL;
    if (n == 0) return RLE_OK;
    const hipStream_t s = (hipStream_t)stream;
    if (n <= kSmallK) {   // one launch, one workgroup
        launch_scan<kSmallThreads>(1u, s, d_gathered, world, n, (n + kSmallThreads - 1) / kSmallThreads, nullptr,
                                   d_offsets);
        return hipGetLastError() == hipSuccess ? RLE_OK : RLE_E_HIP;
    }
    uint32_t items = 0;
    const uint32_t tiles = scan_tiles(n, &items);
    if (!d_ws || ws_bytes < (size_t)tiles * sizeof(int64_t) || ((uintptr_t)d_ws & 7u)) return RLE_E_INVAL;
    int64_t* ws = static_cast<int64_t*>(d_ws);
    hipLaunchKernelGGL(tile_sums_kernel, dim3(tiles), dim3(kScanThreads), 0, s, d_gathered, world, n, items, ws);
    launch_scan<kScanThreads>(tiles, s, d_gathered, world, n, items, ws, d_offsets);
    return hipGetLastError() == hipSuccess ? RLE_OK : RLE_E_HIP;
}

// Whether RCCL resolves in this process (bench.py's preflight: every rank checks before any rank
// enters the blocking communicator init).
extern "C" int rle_dist_available(const char* rccl_path) { return load_rccl(rccl_path) ? RLE_OK : RLE_E_HIP; }

extern "C" int rle_dist_unique_id(void* out, size_t len, const char* rccl_path) {
    if (!out || len < sizeof(ncclUniqueId)) return RLE_E_INVAL;
    if (!load_rccl(rccl_path)) return RLE_E_HIP;
    ncclUniqueId id;
    if (g_rccl.get_unique_id(&id) != 0) return RLE_E_HIP;
    memcpy(out, &id, sizeof(id));
    return RLE_OK;
}

extern "C" int rle_dist_init(const void* id, size_t len, int rank, int world, const char* rccl_path) {
    if (!id || len < sizeof(ncclUniqueId) || world <= 0 || rank < 0 || rank >= world) return RLE_E_INVAL;
    if (g_comm) return RLE_E_INVAL;   // once per process (rle_dist_finalize first)
    if (!load_rccl(rccl_path)) return RLE_E_HIP;
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof(uid));
    if (g_rccl.comm_init_rank(&g_comm, world, uid, rank) != 0) {
        g_comm = nullptr;
        return RLE_E_HIP;
    }
    g_world = world;
    return RLE_OK;
}

extern "C" int rle_dist_gather_offsets(const int64_t* d_sizes, uint32_t n, int64_t* d_gathered, int64_t* d_offsets,
                                       void* d_ws, size_t ws_bytes, void* stream) {
    if (!g_comm) return RLE_E_INVAL;
    if (!d_sizes || !d_gathered || !d_offsets) return RLE_E_INVAL;
    if (ws_bytes < rle_dist_workspace_bytes(n) || (rle_dist_workspace_bytes(n) && !d_ws)) return RLE_E_INVAL;
    if (g_rccl.all_gather(d_sizes, d_gathered, n, kNcclInt64, g_comm, (hipStream_t)stream) != 0) return RLE_E_HIP;
    return rle_dist_offsets_device(d_gathered, (uint32_t)g_world, n, d_offsets, d_ws, ws_bytes, stream);
}

// The exchange off the codec's stream: recorded after the encode issued on codec_stream so far, run
// on comm_stream (gather + scan into result buffer `slot`), and the codec stream only waits -- right
// here, before it issues the step's decode -- for the exchange of the OTHER slot, issued one call
// earlier: so the sizes vector of that slot may be rewritten by the next step's encode.  The host
// cost is this one call (events created once); the codec stream never waits for the gather it just
// started.  The events belong to the process's one communicator and one stream pair: calls must
// alternate the slots (a repeated slot is RLE_E_INVAL: its codec-stream wait would be on the stale
// other slot while the new encode may overwrite sizes the gather still reads), and the function is
// not thread-safe.
namespace {
hipEvent_t g_ev_enc[2] = {}, g_ev_done[2] = {};
bool g_done_rec[2] = {};
int g_last_slot = -1;
}  // namespace
extern "C" int rle_dist_gather_offsets_async(const int64_t* d_sizes, uint32_t n, int64_t* d_gathered,
                                             int64_t* d_offsets, void* d_ws, size_t ws_bytes, void* codec_stream,
                                             void* comm_stream, int slot) {
    if (!g_comm) return RLE_E_INVAL;
    if (!d_sizes || !d_gathered || !d_offsets || (slot != 0 && slot != 1)) return RLE_E_INVAL;
    // a slot repeated while its previous exchange may still read sizes[slot] (the codec stream would
    // wait only on the other slot's): refused; once that exchange has completed, a repeat is safe
    if (slot == g_last_slot && g_done_rec[slot]) {
        const hipError_t q = hipEventQuery(g_ev_done[slot]);
        if (q != hipSuccess) {
            (void)hipGetLastError();   // (hipErrorNotReady is not an error to report later)
            return RLE_E_INVAL;
        }
    }
    for (int k = 0; k < 2; ++k) {
        if (!g_ev_enc[k] && hipEventCreateWithFlags(&g_ev_enc[k], hipEventDisableTiming) != hipSuccess) return RLE_E_HIP;
        if (!g_ev_done[k] && hipEventCreateWithFlags(&g_ev_done[k], hipEventDisableTiming) != hipSuccess) return RLE_E_HIP;
    }
    const hipStream_t cs = (hipStream_t)codec_stream, xs = (hipStream_t)comm_stream;
    if (hipEventRecord(g_ev_enc[slot], cs) != hipSuccess || hipStreamWaitEvent(xs, g_ev_enc[slot], 0) != hipSuccess)
        return RLE_E_HIP;
    if (const int rc = rle_dist_gather_offsets(d_sizes, n, d_gathered, d_offsets, d_ws, ws_bytes, comm_stream)) return rc;
    if (hipEventRecord(g_ev_done[slot], xs) != hipSuccess) return RLE_E_HIP;
    g_done_rec[slot] = true;
    g_last_slot = slot;
    if (g_done_rec[1 - slot] && hipStreamWaitEvent(cs, g_ev_done[1 - slot], 0) != hipSuccess) return RLE_E_HIP;
    return RLE_OK;
}

extern "C" int rle_dist_finalize(void) {
    for (int k = 0; k < 2; ++k) {
        if (g_ev_enc[k]) (void)hipEventDestroy(g_ev_enc[k]);
        if (g_ev_done[k]) (void)hipEventDestroy(g_ev_done[k]);
        g_ev_enc[k] = g_ev_done[k] = nullptr;
        g_done_rec[k] = false;
    }
    g_last_slot = -1;
    int rc = RLE_OK;
    if (g_comm && g_rccl.comm_destroy(g_comm) != 0) rc = RLE_E_HIP;
    g_comm = nullptr;
    g_world = 0;
    return rc;
}
