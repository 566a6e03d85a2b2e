// rle_fileops.hip — device side of the fused append (RLEappend in
// csrc/rle_dropin.cpp): locating the final run of the decoded old content and building the
// 16-byte splice head the incremental re-encode starts from.
//
// The write path of the reference (src/filesystemApi.c:766-775) decodes the whole stored file,
// appends the new bytes and re-encodes all of it.  The encoder's tokens depend only on runs
// (src/rleCompression.c:13-41: every maximal run of length L is cut into floor((L-1)/9) tokens
// of 9 and one final token of r = L - 9 floor((L-1)/9) in 1..9 bytes), so encode(old ‖ new) is
// encode(old) without its final token, followed by encode(c^r ‖ new), c the last byte of old.
// Only the final run's remainder r has to be known; the old stream's tokens before it are kept.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rle_mi355x.h"

namespace rle {

// Start of the final run of mid[0, U): 1 + the last position whose byte differs from mid[U-1]
// (0 when the whole buffer is one run), as an atomicMax into *start (zeroed by the launcher).
// Threads take 16-byte chunks from the end of the buffer backwards; a wave stops as soon as the
// start already found lies past its next chunk, so only the final run (plus one chunk per
// thread) is read.
__global__ __launch_bounds__(256) void last_run_kernel(const uint8_t* __restrict__ mid, uint64_t U,
                                                       unsigned long long* __restrict__ start) {
    const uint8_t c = mid[U - 1];
    const uint64_t nchunks = (U + 15) / 16;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint32_t cc = 0x01010101u * c;
    for (uint64_t q0 = (uint64_t)blockIdx.x * blockDim.x; q0 < nchunks; q0 += stride) {
        // chunks q0 .. q0+255 of this block cover positions below 16 (nchunks - q0); skip the
        // rest of the walk once the final run is known to start above them
        const uint64_t top = 16 * (nchunks - q0);
        if (__hip_atomic_load(start, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= top) break;
        const uint64_t q = q0 + threadIdx.x;
        if (q >= nchunks) continue;
        const uint64_t chunk = nchunks - 1 - q;
        const uint4 v = *reinterpret_cast<const uint4*>(mid + 16 * chunk);
        const uint32_t w[4] = {v.x ^ cc, v.y ^ cc, v.z ^ cc, v.w ^ cc};
        int last = -1;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const bool ne = ((w[k >> 2] >> (8 * (k & 3))) & 0xFFu) != 0u;
            if (ne && 16 * chunk + (uint64_t)k < U) last = k;
        }
        if (last >= 0) atomicMax(start, (unsigned long long)(16 * chunk + (uint64_t)last + 1));
    }
}

// Splice head: head[0, 16) = (16 - r) filler bytes ‖ c^r, with r = ((U - start) - 1) % 9 + 1.
// The filler alternates c^1, c^2 (adjacent bytes differ, none equals c), so it encodes to
// itself, one single-byte token per byte, and the head's final r bytes start a fresh run:
// encode(head ‖ new) = filler ‖ encode(c^r ‖ new).  res[0] = r, res[1..2] = a copy of the head.
__global__ void splice_head_kernel(const uint8_t* __restrict__ mid, uint64_t U,
                                   const unsigned long long* __restrict__ start, uint8_t* __restrict__ head,
                                   uint64_t* __restrict__ res) {
    const uint32_t lane = threadIdx.x;
    const uint8_t c = mid[U - 1];
    const uint64_t L = U - *start;
    const uint32_t r = (uint32_t)((L - 1) % 9) + 1;
    if (lane < 16) {
        const uint8_t v = lane >= 16 - r ? c : (uint8_t)(c ^ ((lane & 1) ? 2 : 1));
        head[lane] = v;
        reinterpret_cast<uint8_t*>(res + 1)[lane] = v;
    }
    if (lane == 0) res[0] = r;
}

}  // namespace rle

// Both kernels of rle_append_prepare_device, with the run-start accumulator (*d_start, zero on
// entry) and the results (res[0] = r, res[1..2] = head) where the caller wants them (the drop-in
// keeps them inside its single-copy call buffers).  Not in the public headers.
int rle_append_prepare_launch(const void* d_mid, uint64_t U, void* d_head, unsigned long long* d_start,
                              uint64_t* d_res, hipStream_t s) {
    const uint64_t nchunks = (U + 15) / 16;
    uint64_t blocks = (nchunks + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(rle::last_run_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, (const uint8_t*)d_mid, U,
                       d_start);
    hipLaunchKernelGGL(rle::splice_head_kernel, dim3(1), dim3(64), 0, s, (const uint8_t*)d_mid, U, d_start,
                       (uint8_t*)d_head, d_res);
    return hipGetLastError() == hipSuccess ? RLE_OK : RLE_E_HIP;
}

extern "C" int rle_append_prepare_device(const void* d_mid, uint64_t U, void* d_head, uint64_t* d_meta,
                                         void* stream) {
    if (U == 0 || !d_mid || !d_head || !d_meta) return RLE_E_INVAL;
    hipStream_t s = (hipStream_t)stream;
    if (hipMemsetAsync(d_meta, 0, sizeof(uint64_t), s) != hipSuccess) return RLE_E_HIP;
    return rle_append_prepare_launch(d_mid, U, d_head, reinterpret_cast<unsigned long long*>(d_meta), d_meta + 1, s);
}
