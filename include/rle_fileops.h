/*
 * rle_fileops.h — the codec operations the reference server's callers compose, fused or batched
 * on the GPU.  C99, plain pointers and sizes; exported by
 * librle_mi355x.so next to the drop-in RLEcompress / RLEdecompress of rleCompression.h.  Same
 * threading, device and no-CPU-path rules as those (include/rleCompression.h).
 *
 *  - RLEappend (f1) replaces the write path's decode ‖ append ‖ re-encode,
 *    src/filesystemApi.c:766-775:
 *        d = RLEdecompress(content, contentSize, uncompressedSize, newContentLen);
 *        memcpy(d + uncompressedSize, newContent, newContentLen);
 *        out = RLEcompress(d, uncompressedSize + newContentLen, &newCompressedSize); free(d);
 *    in one device round trip.  Returns what `out` would be (a malloc block: C' token bytes plus
 *    at least 2 zero bytes; *newCompressedSize = C'), NULL only on allocation failure or, with
 *    errno = EFBIG, for content past RLE_MAX_BUFFER_BYTES (2 GiB).  The old
 *    stream's tokens before its final one are kept and only c^r ‖ newContent is re-encoded (r <= 9,
 *    rle_mi355x.h rle_append_prepare_device), which equals the reference result whenever `content`
 *    is encoder output — the only content the server stores (filesystemApi.c:774 -> :812; a new
 *    file starts empty, :351).  Streams detected as not encoder output (invalid counts, output
 *    past U or short of it, a final token that disagrees with the decoded tail) are re-encoded
 *    whole, as the reference does; other hand-made streams keep their non-canonical prefix.
 *
 *  - RLEdecompressN (f2, f4) decodes n stored files in one launch: readNFilesHandler's loop
 *    (src/filesystemApi.c:675-687) and the eviction loop (src/server.c:314-323).  File i is
 *    RLEdecompress(data[i], compressedSize[i], uncompressedSize[i], 0) written into the caller's
 *    buffer out[i] (uncompressedSize[i] bytes; readNFiles can pass its response buffer at the
 *    file's offset and skip the per-file malloc/memcpy/free).  Returns 0, or -1 with errno =
 *    EINVAL (a NULL array) / ENOMEM / EFBIG (a file past RLE_MAX_BUFFER_BYTES, 2 GiB).
 */
#ifndef RLE_FILEOPS_H
#define RLE_FILEOPS_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

char* RLEappend(char* content, size_t contentSize, size_t uncompressedSize, const char* newContent,
                size_t newContentLen, size_t* newCompressedSize);

int RLEdecompressN(size_t n, char* const* data, const size_t* compressedSize, const size_t* uncompressedSize,
                   char* const* out);

#ifdef __cplusplus
}
#endif

#endif
