"""ctypes binding of librle_mi355x.so — the MI355X RLE block codec.

Mirrors the reference codec interface (samul-1/C-FileStorage-Server-and-Client
include/rleCompression.h:4-5, src/rleCompression.c:9-62): `compress` / `decompress`
call the drop-in RLEcompress / RLEdecompress exactly as src/filesystemApi.c does, and the
`*_batch` functions expose the batched device-resident API of include/rle_mi355x.h on
torch device tensors (PyTorch is only the allocator/stream plumbing here).

The library is required: there is no Python or CPU fallback.  Loading fails loudly when
librle_mi355x.so has not been built (`python -c "import __graft_entry__ as g; g.build()"`).
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "librle_mi355x.so")
# A/B experiments only (tools/ab.sh): load an experimental build instead of the product library
LIB_PATH = os.environ.get("RLE_MI355X_LIB", LIB_PATH)
INCLUDE_DIR = os.path.join(os.path.dirname(HERE), "include")

RLE_OK = 0
RLE_STATUS_OK = 0
RLE_STATUS_OVERFLOW = 1
RLE_STATUS_MISALIGNED = 2
RLE_STATUS_SERIAL = 0x100
RLE_STATUS_SHORT = 0x400
RLE_STATUS_INTERNAL = 0x800
RLE_LAUNCH_STATUS_FLAG = 2

_u64p = ctypes.c_void_p
_lib = None
_libc = ctypes.CDLL("libc.so.6")
_libc.free.argtypes = [ctypes.c_void_p]


class RLEError(RuntimeError):
    pass


class DropinStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in ("calls_compress", "calls_decompress", "bytes_in", "bytes_out",
                                               "bytes_h2d", "bytes_d2h", "ns_stage_in", "ns_device",
                                               "ns_stage_out", "calls_append", "calls_coalesced",
                                               "launches_coalesced", "calls_registered", "calls_reg_fallback")]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


def lib():
    """Load (once) and return the codec library."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RLEError(f"{LIB_PATH} is missing: the HIP codec has not been built")
    L = ctypes.CDLL(LIB_PATH, use_errno=True)   # errno of the drop-in calls (ENOMEM, EFBIG, EINVAL)
    vp, u32, sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_size_t
    L.rle_max_compressed_size.restype = sz
    L.rle_max_compressed_size.argtypes = [sz]
    L.rle_encode_batch_device.restype = ctypes.c_int
    L.rle_encode_batch_device.argtypes = [vp, vp, vp, vp, vp, vp, vp, u32, vp]
    L.rle_decode_batch_device.restype = ctypes.c_int
    L.rle_decode_batch_device.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, u32, vp]
    u64 = ctypes.c_uint64
    L.rle_encode_batch_device_sized.restype = ctypes.c_int
    L.rle_encode_batch_device_sized.argtypes = [vp, vp, vp, vp, vp, vp, vp, u32, u64, vp]
    if hasattr(L, "rle_encode_stream_launch"):   # the RLE_VARIANTS test library only (round 5)
        L.rle_encode_stream_launch.argtypes = [vp, vp, vp, vp, vp, vp, vp, u32, u32, vp]
        L.rle_mi355x_set_stream_waves.argtypes = [ctypes.c_int]
    L.rle_decode_batch_device_sized.restype = ctypes.c_int
    L.rle_decode_batch_device_sized.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, u32, u64, u64, vp]
    L.rle_encode_batch_device_sized_flags.restype = ctypes.c_int
    L.rle_encode_batch_device_sized_flags.argtypes = [vp, vp, vp, vp, vp, vp, vp, u32, u64, u32, vp]
    L.rle_decode_batch_device_sized_flags.restype = ctypes.c_int
    L.rle_decode_batch_device_sized_flags.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, u32, u64, u64, u32, vp]
    L.rle_seg_workspace_bytes.restype = sz
    L.rle_seg_workspace_bytes.argtypes = [u32, ctypes.c_uint64]
    L.rle_encode_batch_device_seg.restype = ctypes.c_int
    L.rle_encode_batch_device_seg.argtypes = [vp, vp, vp, vp, vp, vp, vp, u32, ctypes.c_uint64, vp, sz, vp]
    L.rle_decode_batch_device_seg.restype = ctypes.c_int
    L.rle_decode_batch_device_seg.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, u32, ctypes.c_uint64, vp, sz, vp]
    L.rle_gen_synthetic_device.restype = ctypes.c_int
    L.rle_gen_synthetic_device.argtypes = [vp, vp, vp, vp, vp, u32, vp]
    L.rle_mi355x_selftest.restype = ctypes.c_int
    L.rle_mi355x_selftest.argtypes = []
    L.rle_mi355x_device_count.restype = ctypes.c_int
    L.rle_mi355x_device_count.argtypes = []
    L.rle_mi355x_version.restype = ctypes.c_char_p
    L.rle_mi355x_version.argtypes = []
    L.rle_mi355x_dropin_stats.restype = ctypes.c_int
    L.rle_mi355x_dropin_stats.argtypes = [ctypes.POINTER(DropinStats), ctypes.c_int]
    L.RLEcompress.restype = ctypes.c_void_p
    L.RLEcompress.argtypes = [ctypes.c_char_p, sz, ctypes.POINTER(sz)]
    L.RLEdecompress.restype = ctypes.c_void_p
    L.RLEdecompress.argtypes = [ctypes.c_char_p, sz, sz, sz]
    L.RLEappend.restype = ctypes.c_void_p
    L.RLEappend.argtypes = [ctypes.c_char_p, sz, sz, ctypes.c_char_p, sz, ctypes.POINTER(sz)]
    L.RLEdecompressN.restype = ctypes.c_int
    L.RLEdecompressN.argtypes = [sz, vp, vp, vp, vp]
    L.rle_append_prepare_device.restype = ctypes.c_int
    L.rle_append_prepare_device.argtypes = [vp, ctypes.c_uint64, vp, vp, vp]
    L.rle_mi355x_set_coop_mode.restype = ctypes.c_int
    L.rle_mi355x_set_coop_mode.argtypes = [ctypes.c_int]
    L.rle_decode_release_stream.restype = ctypes.c_int
    L.rle_decode_release_stream.argtypes = [vp]
    L.rle_mi355x_set_dec_round.restype = ctypes.c_int
    L.rle_mi355x_set_dec_round.argtypes = [ctypes.c_int]
    L.rle_copy_device.restype = ctypes.c_int
    L.rle_copy_device.argtypes = [vp, vp, ctypes.c_uint64, vp]
    L.rle_decode_pattern_device.restype = ctypes.c_int
    L.rle_decode_pattern_device.argtypes = [vp] * 6 + [ctypes.c_uint32, vp]
    for f, a in (("rle_dist_available", [ctypes.c_char_p]),
                 ("rle_dist_unique_id", [vp, sz, ctypes.c_char_p]),
                 ("rle_dist_init", [vp, sz, ctypes.c_int, ctypes.c_int, ctypes.c_char_p]),
                 ("rle_dist_gather_offsets", [vp, u32, vp, vp, vp, sz, vp]),
                 ("rle_dist_gather_offsets_async", [vp, u32, vp, vp, vp, sz, vp, vp, ctypes.c_int]),
                 ("rle_dist_offsets_device", [vp, u32, u32, vp, vp, sz, vp]),
                 ("rle_dist_finalize", [])):
        getattr(L, f).restype = ctypes.c_int
        getattr(L, f).argtypes = a
    L.rle_dist_workspace_bytes.restype = sz
    L.rle_dist_workspace_bytes.argtypes = [u32]
    _lib = L
    return L


def max_compressed_size(U: int) -> int:
    return int(lib().rle_max_compressed_size(U))


def round16(x: int) -> int:
    return (x + 15) & ~15


# ------------------------------------------------------------------ drop-in (host) API
def compress(data: bytes) -> bytes:
    """RLEcompress (src/rleCompression.c:9-45) through the drop-in C ABI."""
    c = ctypes.c_size_t(0)
    p = lib().RLEcompress(data, len(data), ctypes.byref(c))
    if not p:
        raise MemoryError("RLEcompress returned NULL")
    out = ctypes.string_at(p, c.value) if c.value else b""
    _libc.free(p)
    return out


def decompress(stream: bytes, U: int, E: int = 0) -> bytes:
    """RLEdecompress (src/rleCompression.c:47-62): U decoded bytes followed by E zero bytes."""
    p = lib().RLEdecompress(stream, len(stream), U, E)
    if not p:
        raise MemoryError("RLEdecompress returned NULL")
    out = ctypes.string_at(p, U + E) if U + E else b""
    _libc.free(p)
    return out


def append(content: bytes, U: int, new: bytes) -> bytes:
    """RLEappend (include/rle_fileops.h): the write path of src/filesystemApi.c:766-775
    -- decode(content, U) ‖ new, re-encoded -- as one fused device round trip."""
    c = ctypes.c_size_t(0)
    p = lib().RLEappend(content, len(content), U, new, len(new), ctypes.byref(c))
    if not p:
        raise MemoryError("RLEappend returned NULL")
    out = ctypes.string_at(p, c.value) if c.value else b""
    _libc.free(p)
    return out


def decompress_n(streams, usizes):
    """RLEdecompressN (include/rle_fileops.h): the n decodes of readNFiles
    (src/filesystemApi.c:675-687) / eviction (src/server.c:314-323) in one launch, into caller buffers."""
    n = len(streams)
    if n != len(usizes):
        raise ValueError("streams and usizes differ in length")
    keep = [ctypes.create_string_buffer(s, len(s) + 1) for s in streams]
    outs = [ctypes.create_string_buffer(max(int(u), 1)) for u in usizes]
    data = (ctypes.c_void_p * max(n, 1))(*[ctypes.addressof(b) for b in keep])
    cs = (ctypes.c_size_t * max(n, 1))(*[len(s) for s in streams])
    us = (ctypes.c_size_t * max(n, 1))(*[int(u) for u in usizes])
    op = (ctypes.c_void_p * max(n, 1))(*[ctypes.addressof(b) for b in outs])
    rc = lib().RLEdecompressN(n, data, cs, us, op)
    if rc != 0:
        raise RLEError(f"RLEdecompressN failed (errno {ctypes.get_errno()})")
    return [o.raw[:int(u)] for o, u in zip(outs, usizes)]


# ------------------------------------------------------------------ batch layout helpers
def layout(sizes, align=16, pad=0):
    """Offsets of buffers packed back to back, each start 16-byte aligned (plus `pad` spare bytes
    after each buffer); returns (offs, total)."""
    offs, pos = [], 0
    for s in sizes:
        offs.append(pos)
        pos += (int(s) + align - 1) // align * align + pad
    return offs, max(pos, align)


def compressed_slots(sizes, pad=0):
    """Worst-case-capacity output slots for encoding buffers of the given sizes."""
    return layout([max_compressed_size(int(s)) for s in sizes], pad=pad)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


STREAM_PER_THREAD = 2   # hipStreamPerThread ((hipStream_t)2, hip_runtime_api.h)


def _stream_ptr(stream):
    if stream is None:
        import torch
        stream = torch.cuda.current_stream()
    if isinstance(stream, int):   # a raw handle (tests: hipStreamPerThread)
        return ctypes.c_void_p(stream)
    return ctypes.c_void_p(stream.cuda_stream)


def release_stream(stream):
    """Free the issue-order array the library keeps for `stream` (rle_decode_release_stream)."""
    _check(lib().rle_decode_release_stream(_stream_ptr(stream)), "rle_decode_release_stream")


def encode_batch(d_in, in_off, in_len, d_out, out_off, out_len, status=None, stream=None, max_len=None, flags=0):
    """Batched encode on device tensors (uint8 data; int64 offsets/lengths; int32 status).  With
    max_len (>= every in_len) the sized entry point runs, which takes the cooperative kernels for
    batches of small buffers; flags (RLE_LAUNCH_STATUS_FLAG) selects the *_sized_flags form."""
    n = in_off.numel()
    if flags:
        rc = lib().rle_encode_batch_device_sized_flags(_ptr(d_in), _ptr(in_off), _ptr(in_len), _ptr(d_out),
                                                       _ptr(out_off), _ptr(out_len), _ptr(status), n,
                                                       int(max_len), int(flags), _stream_ptr(stream))
    elif max_len is None:
        rc = lib().rle_encode_batch_device(_ptr(d_in), _ptr(in_off), _ptr(in_len), _ptr(d_out), _ptr(out_off),
                                           _ptr(out_len), _ptr(status), n, _stream_ptr(stream))
    else:
        rc = lib().rle_encode_batch_device_sized(_ptr(d_in), _ptr(in_off), _ptr(in_len), _ptr(d_out), _ptr(out_off),
                                                 _ptr(out_len), _ptr(status), n, int(max_len), _stream_ptr(stream))
    if rc != RLE_OK:
        raise RLEError(f"rle_encode_batch_device failed: {rc}")


def encode_batch_stream(d_in, in_off, in_len, d_out, out_off, out_len, status=None, stream=None, flags=0):
    """Batched encode, one workgroup per buffer walking it in rounds of tiles (csrc/rle_coop.hip
    enc_stream_body): every input byte read once, any buffer size.  Round 5, measured no faster than
    the segmented encode: in the RLE_VARIANTS test library only (RLE_MI355X_LIB)."""
    rc = lib().rle_encode_stream_launch(_ptr(d_in), _ptr(in_off), _ptr(in_len), _ptr(d_out), _ptr(out_off),
                                        _ptr(out_len), _ptr(status), in_off.numel(), int(flags), _stream_ptr(stream))
    if rc != RLE_OK:
        raise RLEError(f"rle_encode_stream_launch failed: {rc}")


def set_stream_waves(w):
    """Tests: waves per workgroup of the one-pass kernels (4, 8 or 16)."""
    if lib().rle_mi355x_set_stream_waves(int(w)) != RLE_OK:
        raise RLEError(f"set_stream_waves({w})")


def decode_batch(d_in, in_off, in_len, d_out, out_off, out_len, out_cap=None, status=None, stream=None,
                 max_in_len=None, max_out_len=None, flags=0):
    """Batched decode on device tensors.  With max_in_len / max_out_len (>= every in_len / out_len)
    the sized entry point runs (cooperative kernels for batches of small buffers); flags
    (RLE_LAUNCH_STATUS_FLAG) selects the *_sized_flags form."""
    n = in_off.numel()
    if flags:
        rc = lib().rle_decode_batch_device_sized_flags(_ptr(d_in), _ptr(in_off), _ptr(in_len), _ptr(d_out),
                                                       _ptr(out_off), _ptr(out_len), _ptr(out_cap), _ptr(status), n,
                                                       int(max_in_len), int(max_out_len), int(flags),
                                                       _stream_ptr(stream))
    elif max_in_len is None or max_out_len is None:
        rc = lib().rle_decode_batch_device(_ptr(d_in), _ptr(in_off), _ptr(in_len), _ptr(d_out), _ptr(out_off),
                                           _ptr(out_len), _ptr(out_cap), _ptr(status), n, _stream_ptr(stream))
    else:
        rc = lib().rle_decode_batch_device_sized(_ptr(d_in), _ptr(in_off), _ptr(in_len), _ptr(d_out), _ptr(out_off),
                                                 _ptr(out_len), _ptr(out_cap), _ptr(status), n, int(max_in_len),
                                                 int(max_out_len), _stream_ptr(stream))
    if rc != RLE_OK:
        raise RLEError(f"rle_decode_batch_device failed: {rc}")


def seg_workspace(n: int, total_in_bytes: int, device=None):
    """A device workspace for the segmented entry points (caller-owned, reusable across calls on
    one stream)."""
    import torch
    nb = int(lib().rle_seg_workspace_bytes(n, int(total_in_bytes)))
    return torch.empty(nb + 256, dtype=torch.uint8, device=device if device is not None else "cuda")


def _ws_ptr(ws):
    a = ws.data_ptr()
    return ctypes.c_void_p((a + 255) & ~255), ws.numel() - ((-a) & 255)


def encode_batch_seg(d_in, in_off, in_len, d_out, out_off, out_len, status=None, total_in_bytes=None,
                     workspace=None, stream=None):
    """Segmented batched encode (several waves per buffer; for large buffers)."""
    n = in_off.numel()
    total = int(in_len.sum().item()) if total_in_bytes is None else int(total_in_bytes)
    ws = workspace if workspace is not None else seg_workspace(n, total, d_in.device)
    wp, wn = _ws_ptr(ws)
    rc = lib().rle_encode_batch_device_seg(_ptr(d_in), _ptr(in_off), _ptr(in_len), _ptr(d_out), _ptr(out_off),
                                           _ptr(out_len), _ptr(status), n, total, wp, wn, _stream_ptr(stream))
    if rc != RLE_OK:
        raise RLEError(f"rle_encode_batch_device_seg failed: {rc}")


def decode_batch_seg(d_in, in_off, in_len, d_out, out_off, out_len, out_cap=None, status=None,
                     total_in_bytes=None, workspace=None, stream=None):
    """Segmented batched decode (several waves per buffer; for large buffers)."""
    n = in_off.numel()
    total = int(in_len.sum().item()) if total_in_bytes is None else int(total_in_bytes)
    ws = workspace if workspace is not None else seg_workspace(n, total, d_in.device)
    wp, wn = _ws_ptr(ws)
    rc = lib().rle_decode_batch_device_seg(_ptr(d_in), _ptr(in_off), _ptr(in_len), _ptr(d_out), _ptr(out_off),
                                           _ptr(out_len), _ptr(out_cap), _ptr(status), n, total, wp, wn,
                                           _stream_ptr(stream))
    if rc != RLE_OK:
        raise RLEError(f"rle_decode_batch_device_seg failed: {rc}")


def gen_synthetic(d_out, off, length, kind=None, index=None, stream=None):
    n = off.numel()
    rc = lib().rle_gen_synthetic_device(_ptr(d_out), _ptr(off), _ptr(length), _ptr(kind), _ptr(index), n,
                                        _stream_ptr(stream))
    if rc != RLE_OK:
        raise RLEError(f"rle_gen_synthetic_device failed: {rc}")


def copy_device(dst, src, nbytes, stream=None):
    """rle_copy_device: the hand-written 16-byte-per-lane streaming copy bench.py times as the
    practical HBM ceiling (not part of the codec).  nbytes must be a multiple of 16."""
    rc = lib().rle_copy_device(_ptr(dst), _ptr(src), int(nbytes), _stream_ptr(stream))
    if rc != RLE_OK:
        raise RLEError(f"rle_copy_device failed: {rc}")


def decode_pattern(d_in, in_offs, in_lens, d_out, out_offs, out_lens, stream=None):
    """rle_decode_pattern_device: the large-batch decode's memory traffic (tiles of C in, U out, one
    wave per buffer, the decode's occupancy and issue order) without its token work; bench.py times
    it as the ceiling of that access pattern.  Not a decode: d_out receives the tiles' bytes."""
    rc = lib().rle_decode_pattern_device(_ptr(d_in), _ptr(in_offs), _ptr(in_lens), _ptr(d_out), _ptr(out_offs),
                                         _ptr(out_lens), in_offs.numel(), _stream_ptr(stream))
    if rc != RLE_OK:
        raise RLEError(f"rle_decode_pattern_device failed: {rc}")


def set_coop_mode(mode: int):
    """Tests: the cooperative small-buffer kernels never (0), always when the sizes qualify (1), or
    when the launch is resident at once (-1, the default; RLE_MI355X_COOP sets it at load)."""
    if lib().rle_mi355x_set_coop_mode(int(mode)) != RLE_OK:
        raise RLEError(f"bad cooperative mode {mode}")


def set_dec_round(waves: int) -> int:
    """Waves per workgroup of the large-batch decode in rounds (csrc/rle_round.h): 0 off, 4, 8 or
    16 (RLE_MI355X_DEC_ROUND sets it at load); -1 only reads.  Returns the previous setting."""
    rc = lib().rle_mi355x_set_dec_round(int(waves))
    if rc < 0:
        raise RLEError(f"bad decode round width {waves}")
    return rc


def selftest() -> int:
    return int(lib().rle_mi355x_selftest())


def device_count() -> int:
    return int(lib().rle_mi355x_device_count())


def version() -> str:
    return lib().rle_mi355x_version().decode()


def dropin_stats(reset=False) -> dict:
    """Host-path accounting of the drop-in calls made in this process (include/rle_mi355x.h)."""
    st = DropinStats()
    rc = lib().rle_mi355x_dropin_stats(ctypes.byref(st), 1 if reset else 0)
    if rc != RLE_OK:
        raise RLEError(f"rle_mi355x_dropin_stats failed: {rc}")
    return st.as_dict()


# ------------------------------------------------------------------ multi-GPU exchange (csrc/rle_dist.hip)
def _check(rc, what):
    if rc != RLE_OK:
        raise RLEError(f"{what} failed: {rc}")


def _torch_rccl_path():
    """torch's own librccl (the copy torch.distributed's "nccl" backend loaded), so the exchange uses
    the same RCCL library as the process group."""
    import torch
    p = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    return p.encode() if os.path.exists(p) else None


def dist_available():
    """Raises unless RCCL resolves in this process (the preflight of shard.NativeExchange)."""
    _check(lib().rle_dist_available(_torch_rccl_path()), "rle_dist_available")


def dist_unique_id() -> bytes:
    buf = ctypes.create_string_buffer(128)
    _check(lib().rle_dist_unique_id(buf, 128, _torch_rccl_path()), "rle_dist_unique_id")
    return buf.raw


def dist_init(uid: bytes, rank: int, world: int):
    _check(lib().rle_dist_init(uid, len(uid), rank, world, _torch_rccl_path()), "rle_dist_init")


def dist_workspace(n: int, device):
    """The scan workspace of one exchange of n sizes per rank (rle_dist_workspace_bytes): an int64
    device tensor (at least one element), to be kept alive as long as any call or graph uses it.
    Exchanges that may run at once need one each."""
    words = max(1, int(lib().rle_dist_workspace_bytes(int(n))) // 8)
    import torch
    return torch.empty(words, dtype=torch.int64, device=device)


def _ws(ws):
    return (_ptr(ws), ws.numel() * ws.element_size()) if ws is not None else (None, 0)


# Workspaces made for calls that pass none: the scan kernels run on `stream` (or the
# comm stream, or a captured graph replays them) after the call returns, so a temporary torch tensor
# could be handed to another tensor by the caching allocator while they still use it.  One workspace
# per (device, stream, slot) instead, kept for the life of the process: calls on one stream run in
# order, and calls that may run at once (different streams or slots) get different workspaces.  It
# grows when a larger n needs more (keyed on n as well, callers whose n changed from step
# to step grew device memory without bound); the replaced tensor is marked as used by the stream
# (record_stream), so the allocator hands it out again only after the work issued on it so far.
_WS_CACHE = {}


def _default_ws(n, device, stream, slot):
    import torch
    dev = torch.device(device)
    key = (dev.type, dev.index, _stream_ptr(stream).value or 0, slot)
    need = max(1, int(lib().rle_dist_workspace_bytes(int(n))) // 8)
    ws = _WS_CACHE.get(key)
    if ws is None or ws.numel() < need:
        if ws is not None:
            s = stream if isinstance(stream, torch.cuda.Stream) else torch.cuda.current_stream(dev)
            ws.record_stream(s)
        ws = _WS_CACHE[key] = dist_workspace(n, dev)
    return ws


def dist_gather_offsets(sizes, gathered, offsets, stream=None, ws=None):
    """One exchange step (rle_dist_gather_offsets) on `stream`: sizes (int64[n], device) all-gathered
    and scanned into offsets (int64[world * n]) in the global stream order; ws: dist_workspace(n)
    (None: a workspace of this module's own for this stream, kept alive, _default_ws)."""
    if ws is None:
        ws = _default_ws(sizes.numel(), sizes.device, stream, "gather")
    _check(lib().rle_dist_gather_offsets(_ptr(sizes), sizes.numel(), _ptr(gathered), _ptr(offsets), *_ws(ws),
                                         _stream_ptr(stream)), "rle_dist_gather_offsets")


def dist_gather_offsets_async(sizes, gathered, offsets, codec_stream, comm_stream, slot: int, ws=None):
    """The exchange on comm_stream after the work issued on codec_stream (rle_dist_gather_offsets_async);
    codec_stream waits only for the previous call's exchange (the other slot).  Slots must alternate;
    ws: this slot's dist_workspace(n) (None: this module's own for the comm stream and slot)."""
    if ws is None:
        ws = _default_ws(sizes.numel(), sizes.device, comm_stream, ("async", int(slot)))
    _check(lib().rle_dist_gather_offsets_async(_ptr(sizes), sizes.numel(), _ptr(gathered), _ptr(offsets), *_ws(ws),
                                               _stream_ptr(codec_stream), _stream_ptr(comm_stream), int(slot)),
           "rle_dist_gather_offsets_async")


def dist_offsets(gathered, world: int, n: int, offsets, stream=None, ws=None):
    if ws is None:
        ws = _default_ws(n, gathered.device, stream, "offsets")
    _check(lib().rle_dist_offsets_device(_ptr(gathered), world, n, _ptr(offsets), *_ws(ws), _stream_ptr(stream)),
           "rle_dist_offsets_device")


def dist_finalize():
    _check(lib().rle_dist_finalize(), "rle_dist_finalize")
