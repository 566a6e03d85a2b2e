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

// One workgroup: thread t owns a contiguous range of the global order, sums it (gathered is rank
// major: global i = k * world + r sits at gathered[r * n + k]), the workgroup scans the sums in
// LDS, and each thread writes its range's exclusive offsets.
constexpr unsigned kScanThreads = 1024;
__global__ __launch_bounds__(kScanThreads) void offsets_kernel(const int64_t* __restrict__ gathered, uint32_t world,
                                                               uint32_t n, int64_t* __restrict__ out) {
    __shared__ int64_t part[kScanThreads];
    const uint64_t m = (uint64_t)world * n;
    const uint64_t per = (m + kScanThreads - 1) / kScanThreads;
    const uint64_t lo = per * threadIdx.x, hi = lo + per < m ? lo + per : m;
    int64_t s = 0;
    for (uint64_t i = lo; i < hi; ++i) s += gathered[(i % world) * n + i / world];
    part[threadIdx.x] = s;
    __syncthreads();
    for (unsigned d = 1; d < kScanThreads; d <<= 1) {   // inclusive Hillis-Steele scan of the sums
        const int64_t v = threadIdx.x >= d ? part[threadIdx.x - d] : 0;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    int64_t run = threadIdx.x ? part[threadIdx.x - 1] : 0;
    for (uint64_t i = lo; i < hi; ++i) {
        const int64_t v = gathered[(i % world) * n + i / world];
        out[i] = run;
        run += v;
    }
}

}  // namespace

extern "C" int rle_dist_offsets_device(const int64_t* d_gathered, uint32_t world, uint32_t n, int64_t* d_offsets,
                                       void* stream) {
    if (!d_gathered || !d_offsets || world == 0) return RLE_E_INVAL;
    if (n == 0) return RLE_OK;
    hipLaunchKernelGGL(offsets_kernel, dim3(1), dim3(kScanThreads), 0, (hipStream_t)stream, d_gathered, world, n,
                       d_offsets);
    return hipGetLastError() == hipSuccess ? RLE_OK : RLE_E_HIP;
}

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
                                       void* stream) {
    if (!g_comm) return RLE_E_INVAL;
    if (!d_sizes || !d_gathered || !d_offsets) return RLE_E_INVAL;
    if (g_rccl.all_gather(d_sizes, d_gathered, n, kNcclInt64, g_comm, (hipStream_t)stream) != 0) return RLE_E_HIP;
    return rle_dist_offsets_device(d_gathered, (uint32_t)g_world, n, d_offsets, stream);
}

extern "C" int rle_dist_finalize(void) {
    int rc = RLE_OK;
    if (g_comm && g_rccl.comm_destroy(g_comm) != 0) rc = RLE_E_HIP;
    g_comm = nullptr;
    g_world = 0;
    return rc;
}
