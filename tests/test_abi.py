"""CPU tests of the drop-in boundary: librle_mi355x.so loads and exports every function the
headers in include/ declare; the drop-in header is plain C99 (as the reference's callers compile
it, Makefile:6) and declares the reference prototypes (include/rleCompression.h:4-5)."""
import ctypes
import errno
import os
import re
import subprocess
import tempfile

import pytest

import rle_mi355x as R

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(REPO, "include")


def declared_functions():
    names = set()
    for fn in os.listdir(INC):
        if not fn.endswith(".h"):
            continue
        src = open(os.path.join(INC, fn)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        src = re.sub(r"//[^\n]*", "", src)
        for m in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b([A-Za-z_]\w*)\s*\([^;{]*\)\s*;", src, flags=re.M):
            names.add(m.group(1))
    return names


def test_library_exports_every_declared_symbol():
    L = R.lib()
    names = declared_functions()
    assert {"RLEcompress", "RLEdecompress", "rle_encode_batch_device", "rle_decode_batch_device", "RLEappend",
            "RLEdecompressN", "rle_append_prepare_device"} <= names
    for n in sorted(names):
        assert hasattr(L, n), f"librle_mi355x.so does not export {n}"


def test_host_only_entry_points():
    assert R.max_compressed_size(0) == 0
    assert R.max_compressed_size(1) == 1
    assert R.max_compressed_size(2) == 3
    assert R.max_compressed_size(4096) == 6144
    assert "gfx950" in R.version()
    assert R.device_count() >= 0


def test_oversized_buffers_fail_with_efbig():
    """Past RLE_MAX_BUFFER_BYTES (include/rle_mi355x.h) every drop-in entry fails explicitly
    (NULL / -1, errno EFBIG) before touching the data or the GPU -- never a wrong result."""
    L = ctypes.CDLL(R.lib()._name, use_errno=True)
    big = 0x7FFFFFF0 + 1
    buf = ctypes.create_string_buffer(64)
    c = ctypes.c_size_t(123)
    L.RLEcompress.restype = ctypes.c_void_p
    L.RLEcompress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
    ctypes.set_errno(0)
    assert L.RLEcompress(buf, big, ctypes.byref(c)) is None
    assert ctypes.get_errno() == errno.EFBIG and c.value == 0
    L.RLEdecompress.restype = ctypes.c_void_p
    L.RLEdecompress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t]
    for C, U in ((big, 16), (16, big)):
        ctypes.set_errno(0)
        assert L.RLEdecompress(buf, C, U, 0) is None
        assert ctypes.get_errno() == errno.EFBIG
    L.RLEappend.restype = ctypes.c_void_p
    L.RLEappend.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                            ctypes.POINTER(ctypes.c_size_t)]
    ctypes.set_errno(0)
    c.value = 5
    assert L.RLEappend(buf, 3, big - 1, buf, 2, ctypes.byref(c)) is None
    assert ctypes.get_errno() == errno.EFBIG and c.value == 0
    L.RLEdecompressN.restype = ctypes.c_int
    L.RLEdecompressN.argtypes = [ctypes.c_size_t, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_size_t),
                                 ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_char_p)]
    ptrs = (ctypes.c_char_p * 1)(ctypes.cast(buf, ctypes.c_char_p))
    ctypes.set_errno(0)
    assert L.RLEdecompressN(1, ptrs, (ctypes.c_size_t * 1)(big), (ctypes.c_size_t * 1)(16), ptrs) == -1
    assert ctypes.get_errno() == errno.EFBIG


def test_reference_prototypes_exact():
    src = open(os.path.join(INC, "rleCompression.h")).read()
    assert "char* RLEcompress(char* data, size_t origSize, size_t* compressedSize);" in src
    assert ("char* RLEdecompress(char* data, size_t compressedSize, size_t uncompressedSize, "
            "size_t extraAllocation);") in src


def test_headers_compile_as_c99():
    code = '#include "rleCompression.h"\n#include "rle_mi355x.h"\n#include "rle_fileops.h"\n' \
           'int main(void){size_t c=0;(void)c;' \
           'char*(*f)(char*,size_t,size_t*)=RLEcompress;char*(*g)(char*,size_t,size_t,size_t)=RLEdecompress;' \
           'char*(*a)(char*,size_t,size_t,const char*,size_t,size_t*)=RLEappend;' \
           'int(*n)(size_t,char*const*,const size_t*,const size_t*,char*const*)=RLEdecompressN;' \
           '(void)f;(void)g;(void)a;(void)n;return 0;}\n'
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "t.c")
        open(p, "w").write(code)
        r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-pedantic", "-I", INC, "-c", p, "-o",
                            os.path.join(d, "t.o")], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr


def test_c_caller_links_against_dropin():
    """A C caller shaped like src/filesystemApi.c's write path links against the .so unchanged."""
    code = r'''
#include <stdlib.h>
#include <string.h>
#include "rleCompression.h"
int append(char* content, size_t cs, size_t us, const char* add, size_t n, size_t* newcs, char** out) {
    char* d = RLEdecompress(content, cs, us, n);
    memcpy(d + us, add, n);
    *out = RLEcompress(d, us + n, newcs);
    free(d);
    return 0;
}
int main(void) { return 0; }
'''
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "caller.c")
        open(p, "w").write(code)
        r = subprocess.run(["gcc", "-std=c99", "-Wall", "-I", INC, p, "-o", os.path.join(d, "caller"),
                            R.LIB_PATH, "-Wl,-rpath," + os.path.dirname(R.LIB_PATH)], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr


def test_no_oracle_in_product_library():
    """The product .so must not link or embed the CPU oracle."""
    out = subprocess.run(["nm", "-D", R.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle_" not in out
    ldd = subprocess.run(["ldd", R.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in ldd and "librle_ref" not in ldd


def test_fault_injection_only_in_test_build():
    """The allocation-failure hook (RLE_MI355X_FAIL_ALLOC_ABOVE) is compiled into the test build
    only: a leaked variable in a server's environment cannot make the product library fail."""
    with open(R.LIB_PATH, "rb") as f:
        assert b"RLE_MI355X_FAIL_ALLOC_ABOVE" not in f.read()
    th = os.path.join(os.path.dirname(R.LIB_PATH), "build", "librle_mi355x_testhooks.so")
    with open(th, "rb") as f:
        assert b"RLE_MI355X_FAIL_ALLOC_ABOVE" in f.read()


def test_dist_scan_workspace_is_the_callers():
    """The exchange's scan takes its tile sums in the caller's workspace: the size query
    is host-only, and a missing or too-small workspace is refused before any launch."""
    L = R.lib()
    assert L.rle_dist_workspace_bytes(1) == 0 and L.rle_dist_workspace_bytes(512) == 0
    w = L.rle_dist_workspace_bytes(131072)
    assert w >= 8 and w % 8 == 0
    fake = ctypes.c_void_p(0x1000)   # never dereferenced: the call must fail on the workspace check
    assert L.rle_dist_offsets_device(fake, 8, 131072, fake, None, 0, None) == -1
    assert L.rle_dist_offsets_device(fake, 8, 131072, fake, fake, w - 8, None) == -1


def test_launch_flags_are_validated_before_any_launch():
    """rle_*_batch_device_sized_flags (include/rle_mi355x.h): only RLE_LAUNCH_STATUS_FLAG is a known
    bit, and it needs a status array (the completion words); both are refused on the host."""
    L = R.lib()
    fake = ctypes.c_void_p(0x1000)   # never dereferenced: every call below fails on its arguments
    for flags, st in ((1, fake), (4, fake), (R.RLE_LAUNCH_STATUS_FLAG | 8, fake), (R.RLE_LAUNCH_STATUS_FLAG, None)):
        assert L.rle_encode_batch_device_sized_flags(fake, fake, fake, fake, fake, fake, st, 1, 4096, flags, None) == -1
        assert L.rle_decode_batch_device_sized_flags(fake, fake, fake, fake, fake, fake, None, st, 1, 4096, 4096,
                                                     flags, None) == -1
    # n == 0 is a no-op whatever the pointers
    assert L.rle_encode_batch_device_sized_flags(None, None, None, None, None, None, None, 0, 0, 2, None) == 0
