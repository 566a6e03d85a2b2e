/*
 * rleCompression.h — drop-in replacement header for the MI355X RLE block codec.
 *
 * Declares exactly the two entry points of the reference codec header
 * (samul-1/C-FileStorage-Server-and-Client include/rleCompression.h:4-5), with the same
 * names, C linkage, non-const parameter types and return types, so
 * src/filesystemApi.c (:597, :680, :767, :774) and src/server.c (:317) compile and link
 * against librle_mi355x.so unchanged.  C99, no HIP/C++ types.
 *
 * Contract:
 *  - RLEcompress   replaces src/rleCompression.c:9-45.   Returns a fresh malloc'd block
 *                  (release with free()) holding the C-byte token stream followed by at least
 *                  2 zero bytes; *compressedSize = C is always written.  U = 0 returns a
 *                  non-NULL block and C = 0.  NULL only on allocation failure.
 *  - RLEdecompress replaces src/rleCompression.c:47-62.  Returns a fresh malloc'd block of
 *                  uncompressedSize + extraAllocation bytes: the decoded U bytes followed by
 *                  E zero bytes.  Bytes of `data` past compressedSize are read as 0x00 (the
 *                  zero padding every stored stream carries).  NULL only on allocation failure.
 *  - Both are re-entrant and may be called concurrently from any number of threads; the
 *    device is initialised lazily on the first call.  The codec runs on the GPU only: with
 *    no usable MI355X the library prints a diagnostic and aborts (it has no CPU path).
 */
#ifndef RLE_COMPRESSION_H
#define RLE_COMPRESSION_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

char* RLEcompress(char* data, size_t origSize, size_t* compressedSize);
char* RLEdecompress(char* data, size_t compressedSize, size_t uncompressedSize, size_t extraAllocation);

#ifdef __cplusplus
}
#endif

#endif
