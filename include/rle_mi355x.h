/*
 * rle_mi355x.h — batched, device-resident entry points of the MI355X RLE block codec.
 *
 * These are the batch forms of the reference codec (src/rleCompression.c:9-62, declared at
 * include/rleCompression.h:4-5 of samul-1/C-FileStorage-Server-and-Client): the same token
 * grammar, byte-identical output, applied to B independent buffers in one launch.  The
 * reference has no batch API; its natural batch is readNFilesHandler's decode loop
 * (src/filesystemApi.c:680-687), and the eviction decode loop (src/server.c:314-323).
 *
 * All pointers named d_* are device (HBM) pointers; `stream` is a hipStream_t passed as
 * void* (NULL = the default stream).  Calls are asynchronous on that stream.  Return value:
 * RLE_OK, or a negative RLE_E_* host-side error (nothing was launched).
 *
 * Layout rules:
 *  - buffer i occupies d_in + d_in_off[i] .. + d_in_len[i]; d_in + d_in_off[i] and
 *    d_out + d_out_off[i] must be 16-byte aligned (else d_status[i] = RLE_STATUS_MISALIGNED
 *    and that buffer is skipped);
 *  - encode: the output slot of buffer i must hold rle_max_compressed_size(d_in_len[i])
 *    bytes; exactly d_out_len[i] = C bytes are written;
 *  - decode: d_in_len[i] = C (compressed), d_out_len[i] = U (decoded size, as the reference's
 *    uncompressedSize).  d_out_cap[i] (NULL: = U) is the writable slot size, U <= cap; the
 *    first U bytes are always written.  Bytes of a slot past U are written only for streams
 *    the encoder never emits and only where the reference would write them (its
 *    extraAllocation region).
 */
#ifndef RLE_MI355X_H
#define RLE_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* host-side return codes */
#define RLE_OK          0
#define RLE_E_INVAL    (-1)   /* bad argument */
#define RLE_E_HIP      (-2)   /* a HIP runtime call failed */
#define RLE_E_NODEV    (-3)   /* no usable gfx950 device */

/* Largest buffer (input or decoded) one kernel handles: in-buffer offsets are 32-bit. */
#define RLE_MAX_BUFFER_BYTES 0x7FFFFFF0u

/* per-buffer status bits (d_status[i]) */
#define RLE_STATUS_OK          0u
#define RLE_STATUS_OVERFLOW    1u      /* decode: stream writes past cap (reference: heap overflow); truncated */
#define RLE_STATUS_MISALIGNED  2u      /* input or output slot not 16-byte aligned; buffer skipped */
#define RLE_STATUS_TOOLARGE    4u      /* buffer larger than RLE_MAX_BUFFER_BYTES (2 GiB); buffer skipped */
#define RLE_STATUS_SERIAL      0x100u  /* info: stream decoded by the exact serial path (not encoder output) */
#define RLE_STATUS_SHORT       0x400u  /* info: the stream decodes to fewer than U bytes, the rest is zero
                                          (not encoder output) */
#define RLE_STATUS_INTERNAL    0x800u  /* the segmented kernels' carry wait ran out (never expected): output
                                          not trusted */

/* Worst-case compressed size of U bytes (every run of length 2: 3 bytes per 2 input bytes). */
size_t rle_max_compressed_size(size_t U);

/* Batched encode (RLEcompress, src/rleCompression.c:9-45) of n buffers.
 * d_status may be NULL. */
int rle_encode_batch_device(const void* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                            void* d_out, const uint64_t* d_out_off, uint64_t* d_out_len,
                            uint32_t* d_status, uint32_t n, void* stream);

/* Batched decode (RLEdecompress, src/rleCompression.c:47-62) of n buffers.
 * d_out_cap and d_status may be NULL.  Batches of more than 4096 buffers are issued longest first:
 * a small sort launch writes an issue-order array that the library keeps per (device, stream) and
 * reuses (the first call on a stream allocates it, stream-ordered); calls from several host threads
 * on one stream are serialised while they enqueue. */
int rle_decode_batch_device(const void* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                            void* d_out, const uint64_t* d_out_off, const uint64_t* d_out_len,
                            const uint64_t* d_out_cap, uint32_t* d_status, uint32_t n, void* stream);

/* The same two launches with the batch's largest sizes known on the host (max_in_len >= every
 * d_in_len[i]; decode: max_out_len >= every d_out_len[i]).  Few small buffers (encode:
 * max_in_len <= 8 KiB; decode: max_in_len <= 8064 and max_out_len <= 16 KiB; and no more
 * workgroups than the chip holds at once, from the occupancy API) then run the cooperative
 * kernels, one workgroup per buffer and one wave per tile, so a buffer's tiles run side by side
 * instead of one after another (a single file, a small readN).  Other batches (or
 * RLE_MI355X_COOP=0) take the kernels above.  Output and status are the same bytes. */
int rle_encode_batch_device_sized(const void* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                                  void* d_out, const uint64_t* d_out_off, uint64_t* d_out_len,
                                  uint32_t* d_status, uint32_t n, uint64_t max_in_len, void* stream);
int rle_decode_batch_device_sized(const void* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                                  void* d_out, const uint64_t* d_out_off, const uint64_t* d_out_len,
                                  const uint64_t* d_out_cap, uint32_t* d_status, uint32_t n,
                                  uint64_t max_in_len, uint64_t max_out_len, void* stream);

/* The sized launches with launch flags.  RLE_LAUNCH_STATUS_FLAG (needs d_status): each buffer's
 * status word is stored last, behind a system-scope release of every output byte and d_out_len
 * word of that buffer, so a host that placed d_out / d_status in mapped pinned memory
 * (hipHostMallocMapped) and preset the status words to a value no status takes (e.g. 0xFFFFFFFF)
 * can poll them instead of synchronizing the stream: once a status word changes, the buffer's
 * output is readable from the host.  The drop-in's small zero-copy calls work this way (saves
 * ~4.5 us per call against hipStreamSynchronize, profiles/r4a_sync_probe.txt).  Other flag bits:
 * RLE_E_INVAL. */
#define RLE_LAUNCH_STATUS_FLAG 2u
int rle_encode_batch_device_sized_flags(const void* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                                        void* d_out, const uint64_t* d_out_off, uint64_t* d_out_len,
                                        uint32_t* d_status, uint32_t n, uint64_t max_in_len, uint32_t flags,
                                        void* stream);
int rle_decode_batch_device_sized_flags(const void* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                                        void* d_out, const uint64_t* d_out_off, const uint64_t* d_out_len,
                                        const uint64_t* d_out_cap, uint32_t* d_status, uint32_t n,
                                        uint64_t max_in_len, uint64_t max_out_len, uint32_t flags, void* stream);

/* Synthetic batch generator: xorshift64 (13,7,17), state seed
 * 0x9E3779B97F4A7C15 + index, one step per byte; kind 0 zero, 1 random, 2 runs50,
 * 3 runs90, 4 pairs.  d_kind / d_index may be NULL (kind 1, index = i). */
int rle_gen_synthetic_device(void* d_out, const uint64_t* d_off, const uint64_t* d_len,
                             const uint32_t* d_kind, const uint64_t* d_index, uint32_t n, void* stream);

/* Host-path accounting of the drop-in RLEcompress/RLEdecompress (process-wide): bytes the callers
 * passed in and got back, bytes moved host->device / device->host, and wall time spent staging
 * into pinned memory, on the device round trip (H2D + kernel + D2H, stream-synchronised) and
 * copying out to the caller's malloc block.  reset != 0 zeroes the counters after reading. */
typedef struct {
    uint64_t calls_compress, calls_decompress;
    uint64_t bytes_in, bytes_out, bytes_h2d, bytes_d2h;
    uint64_t ns_stage_in, ns_device, ns_stage_out;
    uint64_t calls_append;   /* RLEappend (include/rle_fileops.h); RLEdecompressN counts per file */
    uint64_t calls_coalesced, launches_coalesced;   /* zero-copy small calls and the combined launches
                                                       they ran in (concurrent callers share one) */
    uint64_t calls_registered;     /* large calls run on the caller's registered memory (RLE_MI355X_REG_MIN) */
    uint64_t calls_reg_fallback;   /* ... and those that took the staging instead (registration refused or
                                      overlapping another call's) */
} rle_dropin_stats_t;
int rle_mi355x_dropin_stats(rle_dropin_stats_t* out, int reset);

/* Runs the cross-lane (DPP) primitive self-test on the current device; 0 = pass. */
int rle_mi355x_selftest(void);

/* Large buffers: the same batched encode / decode with every buffer cut into segments of 4..64
 * tiles of 1008 input bytes (about 16 segments per CU over the batch) processed by separate waves
 * (per-segment summaries, a per-buffer scan of the run / token phase crossing segment boundaries,
 * then per-segment writes: four launches).  Same arguments, results and status codes as
 * rle_encode_batch_device / rle_decode_batch_device, plus:
 *   total_in_bytes  >= the sum of the n input lengths (sizes the segment tables; a buffer whose
 *                   segments do not fit gets RLE_STATUS_TOOLARGE)
 *   d_workspace     caller-owned device memory of at least rle_seg_workspace_bytes(n,
 *                   total_in_bytes) bytes, 256-byte aligned, not used by another launch in flight
 * Use it when buffers are large relative to the batch (one big file, a mixed 4 KiB - 1 MiB batch);
 * RLEcompress / RLEdecompress use it from 48 KiB (encode input) / 32 KiB (decode input).
 * Replaces src/rleCompression.c:9-62 like the entries above. */
size_t rle_seg_workspace_bytes(uint32_t n, uint64_t total_in_bytes);
int rle_encode_batch_device_seg(const void* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                                void* d_out, const uint64_t* d_out_off, uint64_t* d_out_len,
                                uint32_t* d_status, uint32_t n, uint64_t total_in_bytes,
                                void* d_workspace, size_t workspace_bytes, void* stream);
int rle_decode_batch_device_seg(const void* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                                void* d_out, const uint64_t* d_out_off, const uint64_t* d_out_len,
                                const uint64_t* d_out_cap, uint32_t* d_status, uint32_t n,
                                uint64_t total_in_bytes, void* d_workspace, size_t workspace_bytes,
                                void* stream);

/* Fused append, device half (used by RLEappend, include/rle_fileops.h).
 * d_mid holds the decoded old content, U >= 1 bytes, 16-byte aligned.  Finds the final run of
 * d_mid (byte c, length L), r = (L - 1) % 9 + 1 (the size of the reference encoder's last token of
 * that run, src/rleCompression.c:22-39), and writes the 16-byte splice head
 *   d_head[0, 16) = (16 - r) filler bytes ‖ c^r
 * whose filler encodes to itself byte for byte, so encode(head ‖ new) = filler ‖ encode(c^r ‖ new).
 * d_meta (4 u64, device): [0] final run start, [1] r, [2..3] a copy of the head.  Asynchronous on
 * `stream`; RLE_E_INVAL when U == 0. */
int rle_append_prepare_device(const void* d_mid, uint64_t U, void* d_head, uint64_t* d_meta, void* stream);

/* Diagnostic builds only (RLE_STAMPS=1, never the product library): per-segment decode cycle sums
 * over all waves: [tile wait, scan, scatter, flush reads, flush fill, flush store, flush re-zero,
 * move/drain/finish, waves]; RLE_E_INVAL otherwise. */
int rle_mi355x_stamps(unsigned long long* out9, int reset);

/* Diagnostic builds only (RLE_TIMELINE=1, never the product library): per-buffer wave timelines of
 * the one-wave batch kernels, 16384 x 16 u64 (s_memrealtime at entry, walk start, tiles 0..7, end;
 * HW_ID, XCC_ID); RLE_E_INVAL otherwise. */
int rle_mi355x_timeline(unsigned long long* out, int reset);

/* ---- multi-GPU exchange (csrc/rle_dist.hip) -------------------------------
 * The one exchange of a batch sharded round-robin over N GPUs (shard.py, bench.py --gpus N): each
 * rank's per-buffer compressed sizes all-gathered over RCCL and scanned into offsets in the global
 * stream (global buffer i = k * world + r is rank r's k-th buffer).  No reference interface: the
 * reference server is single-host, single-process (src/server.c); this replaces the Python
 * all_gather + cumsum of shard.global_offsets with one host call.  RCCL is resolved at run time from
 * the process's librccl.so.1 (or rccl_path when non-NULL).
 *   rle_dist_unique_id: a communicator id (128 bytes) on one rank, to be broadcast to all ranks.
 *   rle_dist_init: this rank's communicator (once per process).
 *   rle_dist_gather_offsets: on `stream`, after the work issued on it so far: all-gather
 *     d_sizes[n] into d_gathered[world * n] (rank major), then the exclusive scan in global order
 *     into d_offsets[world * n].
 *   rle_dist_offsets_device: the scan alone, on `stream` (tests).  Two launches over the whole
 *     chip, with the tile sums in the caller's workspace d_ws of ws_bytes >=
 *     rle_dist_workspace_bytes(n) bytes (0 for n <= 512: d_ws may be NULL; 8-byte aligned).  Scans
 *     that may run at once need workspaces of their own; a captured graph keeps the pointer, so the
 *     caller keeps the workspace alive while the graph exists.  RLE_E_INVAL when it is too small.
 *   rle_dist_available: RLE_OK when the RCCL symbols resolve in this process (a preflight that every
 *     rank runs before any rank enters the blocking rle_dist_init).
 *   rle_dist_finalize: destroys the communicator. */
int rle_dist_available(const char* rccl_path);
int rle_dist_unique_id(void* out, size_t len, const char* rccl_path);
int rle_dist_init(const void* id, size_t len, int rank, int world, const char* rccl_path);
size_t rle_dist_workspace_bytes(uint32_t n);
int rle_dist_gather_offsets(const int64_t* d_sizes, uint32_t n, int64_t* d_gathered, int64_t* d_offsets, void* d_ws,
                            size_t ws_bytes, void* stream);
int rle_dist_offsets_device(const int64_t* d_gathered, uint32_t world, uint32_t n, int64_t* d_offsets, void* d_ws,
                            size_t ws_bytes, void* stream);
/* rle_dist_gather_offsets off the codec's stream: after the work issued on codec_stream so far, the
 * gather + scan run on comm_stream into the caller's result buffers of `slot` (0 or 1, alternating
 * per step); codec_stream is made to wait only for the previous call's exchange (the other slot),
 * so the caller may rewrite the other slot's sizes in its next step.  Each slot needs its own workspace
 * (d_ws, as rle_dist_gather_offsets).  Calls must alternate the slots (a repeated slot is
 * RLE_E_INVAL); one communicator and one stream pair per process; not thread-safe. */
int rle_dist_gather_offsets_async(const int64_t* d_sizes, uint32_t n, int64_t* d_gathered, int64_t* d_offsets,
                                  void* d_ws, size_t ws_bytes, void* codec_stream, void* comm_stream, int slot);
int rle_dist_finalize(void);

/* Tests: the cooperative mode of the sized entry points, in-process (0 never, 1 whenever the sizes
 * qualify, -1 residency-gated default; RLE_MI355X_COOP sets the initial mode).  RLE_E_INVAL
 * otherwise. */
int rle_mi355x_set_coop_mode(int mode);

/* Tests / A-B: waves per workgroup of the large-batch decode in rounds (0 off, 4, 8 or 16): batches
 * of more than 4096 buffers through the sized entry points whose max_in_len is at least 8 decode
 * tiles (8064 bytes) decode one workgroup per buffer, its waves on consecutive tiles.
 * RLE_MI355X_DEC_ROUND sets the initial value; -1 only reads it.  Returns the previous setting, or
 * RLE_E_INVAL. */
int rle_mi355x_set_dec_round(int waves);

/* Large decodes (more than 4096 buffers) keep their issue-order array per (device, stream handle),
 * up to 16 of them, the least recently used handed over when a new stream needs one; every array
 * is used in turn across the queues a handle may name (hipStreamPerThread, a reused handle).  This
 * frees the array kept for `stream` on the current device, behind the work already issued on it. */
int rle_decode_release_stream(void* stream);

/* Measurement only (not the codec): copies nbytes (a multiple of 16, both pointers 16-byte aligned)
 * from d_src to d_dst on `stream` with a hand-written 16-byte-per-lane streaming kernel; bench.py
 * times it as the practical HBM ceiling of SURVEY.md §8(d).  RLE_E_INVAL on bad sizes. */
int rle_copy_device(void* d_dst, const void* d_src, uint64_t nbytes, void* stream);

/* Measurement only (not the codec): the large-batch decode's memory traffic without its token work:
 * each of the n buffers (decode_batch arguments) read in decode tiles and U bytes written, one wave
 * per buffer, the decode's occupancy and issue order.  bench.py times it beside the north-star decode
 * as the ceiling of that access pattern.  The output bytes are not a decode. */
int rle_decode_pattern_device(const void* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len, void* d_out,
                              const uint64_t* d_out_off, const uint64_t* d_out_len, uint32_t n, void* stream);

/* The drop-in's background start-up (HIP runtime, warm thread contexts) at library load: 1 when this
 * process started it, 0 otherwise.  It starts in a program that links the library (the reference
 * server, INTEGRATION.md §2: the library is among the main program's DT_NEEDED entries) or whenever
 * RLE_MI355X_PREINIT > 0; a process that dlopen()s the library (Python ctypes) does no GPU work
 * before its first codec call unless RLE_MI355X_PREINIT asks for it.  No reference interface. */
int rle_mi355x_preinit_state(void);

/* Number of visible HIP devices (0 when none). */
int rle_mi355x_device_count(void);

const char* rle_mi355x_version(void);

#ifdef __cplusplus
}
#endif
#endif
