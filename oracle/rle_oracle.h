/*
 * rle_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * Clean-room CPU restatement of the reference RLE block codec
 * (samul-1/C-FileStorage-Server-and-Client, src/rleCompression.c:9-62), used as the
 * parity checker for the MI355X HIP codec.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library; the product path
 * (librle_mi355x.so) never links or calls it.
 *
 * Pinned against: the compiled reference (oracle/_ref, built by oracle/Makefile from
 * /root/reference/src/rleCompression.c) on the golden vectors in tests/golden/,
 * the report's KAT (Relazione.pdf p.3: "aaaaaaaaaaaab" -> "aa9aa3b") and the
 * sha256 pins of the reference's own test fixtures.
 */
#ifndef RLE_ORACLE_H
#define RLE_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Decode status codes (shared meaning with include/rle_mi355x.h). */
#define ORACLE_RLE_OK        0u
#define ORACLE_RLE_OVERFLOW  1u   /* the reference would write past its U+E allocation (heap overflow) */

/* Worst-case compressed size of U input bytes (all runs of length 2: floor(1.5 U)). */
size_t oracle_rle_max_compressed(size_t U);

/* Encode x[0,U) into out (capacity >= oracle_rle_max_compressed(U)); returns C.
 * Restates src/rleCompression.c:9-45. */
size_t oracle_rle_encode(const uint8_t* x, size_t U, uint8_t* out);

/* Decode y[0,C) with the reference's exact semantics (src/rleCompression.c:47-62):
 * bytes at index >= C read as 0x00 (the calloc padding of every stream the reference
 * server stores), replicate loop capped at U, every first-byte write unconditional.
 * out must hold `cap` bytes (cap >= U; the reference allocates U+E) and is fully written
 * (untouched bytes are zero, like calloc).  Returns ORACLE_RLE_OK or ORACLE_RLE_OVERFLOW
 * (the reference would overflow its heap block; output truncated at cap). */
uint32_t oracle_rle_decode(const uint8_t* y, size_t C, size_t U, size_t cap, uint8_t* out,
                           size_t* written);

/* Batched helpers (pthreads; nthreads<=0 -> 1). Offsets/lengths are per buffer. */
void oracle_rle_encode_batch(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len,
                             uint8_t* out, const uint64_t* out_off, uint64_t* out_len,
                             uint32_t n, int nthreads);
void oracle_rle_decode_batch(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len,
                             uint8_t* out, const uint64_t* out_off, const uint64_t* out_len,
                             uint32_t* status, uint32_t n, int nthreads);

/* Synthetic inputs: xorshift64 (13,7,17), state seed
 * 0x9E3779B97F4A7C15 + buffer_index, one step per byte.
 * kind: 0 zero, 1 random, 2 runs50, 3 runs90, 4 pairs (worst case, C = 1.5U). */
void oracle_gen_buffer(uint32_t kind, uint64_t index, uint8_t* out, size_t U);

#ifdef __cplusplus
}
#endif
#endif
