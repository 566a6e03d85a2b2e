"""TEST INFRASTRUCTURE ONLY — ctypes binding of the CPU oracle (oracle/librle_oracle.so) and of
the compiled reference (oracle/_ref/librle_ref_O0.so, built from /root/reference by
oracle/Makefile).  Imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
only, as the checker; the product path never loads it.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "librle_oracle.so")
REF_SO = os.path.join(HERE, "_ref", "librle_ref_O0.so")
REF_BENCH = {"O0": os.path.join(HERE, "_ref", "ref_bench_O0"), "O2": os.path.join(HERE, "_ref", "ref_bench_O2")}

_o = None
_r = None
_libc = ctypes.CDLL("libc.so.6")
_libc.free.argtypes = [ctypes.c_void_p]


def oracle():
    global _o
    if _o is None:
        L = ctypes.CDLL(ORACLE_SO)
        vp, sz, u32, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint64
        L.oracle_rle_max_compressed.restype = sz
        L.oracle_rle_max_compressed.argtypes = [sz]
        L.oracle_rle_encode.restype = sz
        L.oracle_rle_encode.argtypes = [ctypes.c_char_p, sz, vp]
        L.oracle_rle_decode.restype = u32
        L.oracle_rle_decode.argtypes = [ctypes.c_char_p, sz, sz, sz, vp, ctypes.POINTER(sz)]
        L.oracle_rle_encode_batch.restype = None
        L.oracle_rle_encode_batch.argtypes = [vp, vp, vp, vp, vp, vp, u32, ctypes.c_int]
        L.oracle_rle_decode_batch.restype = None
        L.oracle_rle_decode_batch.argtypes = [vp, vp, vp, vp, vp, vp, vp, u32, ctypes.c_int]
        L.oracle_gen_buffer.restype = None
        L.oracle_gen_buffer.argtypes = [u32, u64, vp, sz]
        _o = L
    return _o


def encode(x: bytes) -> bytes:
    L = oracle()
    out = ctypes.create_string_buffer(max(1, L.oracle_rle_max_compressed(len(x))))
    c = L.oracle_rle_encode(x, len(x), out)
    return out.raw[:c]


def decode(y: bytes, U: int, cap: int = None):
    """Returns (bytes of length cap, status)."""
    L = oracle()
    cap = U if cap is None else cap
    out = ctypes.create_string_buffer(max(1, cap))
    w = ctypes.c_size_t(0)
    st = L.oracle_rle_decode(y, len(y), U, cap, out, ctypes.byref(w))
    return out.raw[:cap], int(st)


def gen(kind: int, index: int, U: int) -> bytes:
    buf = ctypes.create_string_buffer(max(1, U))
    oracle().oracle_gen_buffer(kind, index, buf, U)
    return buf.raw[:U]


def gen_into(kind: int, index: int, arr_ptr: int, U: int):
    oracle().oracle_gen_buffer(kind, index, ctypes.c_void_p(arr_ptr), U)


def encode_batch_np(inp, in_off, in_len, out, out_off, out_len, nthreads=8):
    """numpy arrays (uint8 data, uint64 offsets/lengths)."""
    oracle().oracle_rle_encode_batch(inp.ctypes.data, in_off.ctypes.data, in_len.ctypes.data, out.ctypes.data,
                                     out_off.ctypes.data, out_len.ctypes.data, len(in_off), nthreads)


def decode_batch_np(inp, in_off, in_len, out, out_off, out_len, status, nthreads=8):
    oracle().oracle_rle_decode_batch(inp.ctypes.data, in_off.ctypes.data, in_len.ctypes.data, out.ctypes.data,
                                     out_off.ctypes.data, out_len.ctypes.data, status.ctypes.data, len(in_off),
                                     nthreads)


def reference():
    """The compiled reference codec (only where oracle/_ref was built)."""
    global _r
    if _r is None:
        L = ctypes.CDLL(REF_SO)
        L.RLEcompress.restype = ctypes.c_void_p
        L.RLEcompress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
        L.RLEdecompress.restype = ctypes.c_void_p
        L.RLEdecompress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t]
        _r = L
    return _r


def ref_compress(x: bytes) -> bytes:
    c = ctypes.c_size_t(0)
    p = reference().RLEcompress(x, len(x), ctypes.byref(c))
    out = ctypes.string_at(p, c.value) if c.value else b""
    _libc.free(p)
    return out


def ref_decompress(y: bytes, U: int, E: int = 0) -> bytes:
    padded = y + b"\0\0\0"
    p = reference().RLEdecompress(padded, len(y), U, E)
    out = ctypes.string_at(p, U + E) if U + E else b""
    _libc.free(p)
    return out
