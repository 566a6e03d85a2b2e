"""GPU parity of the fused / batched file operations (include/rle_fileops.h, SURVEY.md §8 (f1),
(f2), (f4)) against the reference composition they replace, restated with the oracle:

  append   src/filesystemApi.c:766-775   decode(content, U, E=len(new)) ; memcpy at U ; encode(U+len(new))
  readN    src/filesystemApi.c:675-687   RLEdecompress(content_i, C_i, U_i, 0) per file
  evict    src/server.c:314-323          the same decode per victim

Bit-exact everywhere."""
import numpy as np
import pytest

import rle_mi355x as R
import rle_oracle as O

pytestmark = pytest.mark.gpu


def ref_append(content, U, new):
    """src/filesystemApi.c:767-774 with the oracle in place of src/rleCompression.c."""
    d, _ = O.decode(content, U, U + len(new))
    return O.encode(d[:U] + new)


def _runs(rng, n, alpha, maxrun):
    vals = rng.choice(np.frombuffer(alpha, np.uint8), size=n)
    reps = rng.integers(1, maxrun + 1, size=n)
    return np.repeat(vals, reps).tobytes()


def test_append_final_run_remainders():
    # old content ending in a run of every length 1..40 (all remainders r = 1..9, several 9-tokens),
    # appended bytes that continue the run, break it, or are empty
    cases = []
    for ch in (b"a", b"9", b"1", b"\0", b"\xff"):
        for L in range(1, 41):
            old = b"xy" + ch * L
            for new in (b"", ch, ch * 8, ch * 9, ch * 20 + b"z", b"z", b"zz" + ch, bytes(range(50))):
                cases.append((old, new))
    for old, new in cases:
        y = O.encode(old)
        assert R.append(y, len(old), new) == ref_append(y, len(old), new), (old, new)


def test_append_digit_heavy_streams():
    # streams whose bytes are digits, where the final token cannot be found by reading backwards
    rng = np.random.default_rng(11)
    for i in range(400):
        old = _runs(rng, int(rng.integers(1, 60)), b"23456789" if i % 2 else b"99a1", 12)
        new = _runs(rng, int(rng.integers(0, 30)), b"2399", 12)
        y = O.encode(old)
        assert R.append(y, len(old), new) == O.encode(old + new), (old, new)


def test_append_chained_writes_build_the_file():
    # a file written by successive appends, as the server does (a new file starts empty, :351)
    rng = np.random.default_rng(5)
    for kind in range(5):
        content, plain = b"", b""
        for k in range(30):
            n = int(rng.integers(0, 3000))
            new = O.gen(kind, 100 * kind + k, n)
            content = R.append(content, len(plain), new)
            plain += new
            assert content == O.encode(plain), (kind, k)


def test_append_large_and_segmented_sizes():
    for old, new in [(bytes(1 << 20), bytes(5000)), (O.gen(1, 1, 300000), O.gen(2, 2, 200000)),
                     (O.gen(3, 3, 70000), b""), (b"q" * 100001, b"q" * 7), (O.gen(2, 4, 5), O.gen(1, 5, 1 << 20))]:
        y = O.encode(old)
        assert R.append(y, len(old), new) == O.encode(old + new), (len(old), len(new))


def test_append_zero_copy_sizes():
    """The zero-copy append (csrc/rle_dropin.cpp append_small_zc): old streams the one-wave or the
    cooperative decode takes from the mapped buffer (up to 80 tiles decoding to 64 KiB), new bytes
    up to the cooperative encode's 64 KiB, at and around their edges; a stream that is not encoder
    output in that range falls back to the whole re-encode."""
    cases = []
    for kind, U, A in [(1, 4096, 4096), (2, 32000, 100), (1, 33000, 1), (2, 65536, 4096), (3, 65536, 65520),
                       (1, 53000, 60000), (0, 65536, 0), (1, 65536, 65521), (2, 40000, 70000)]:
        cases.append((O.gen(kind, U + A, U), O.gen((kind + 1) % 4, U ^ A, A)))
    for old, new in cases:
        y = O.encode(old)
        assert R.append(y, len(old), new) == O.encode(old + new), (len(old), len(y), len(new))
    # hand-made: a long literal stream whose last token is not the encoder's
    y = O.encode(O.gen(1, 77, 40000))
    bad = y[:-1] + (b"5" if y[-1:] != b"5" else b"6")
    assert R.append(bad, 40000, b"zz") == ref_append(bad, 40000, b"zz")


def test_append_empty_and_not_encoder_streams():
    assert R.append(b"", 0, b"") == b""
    assert R.append(b"", 0, b"aaab") == b"aa3b"
    # no stream but U > 0: the reference decodes U zero bytes (src/rleCompression.c:48)
    assert R.append(b"", 5, b"ab") == ref_append(b"", 5, b"ab")
    # hand-made streams the encoder never emits: non-canonical final token, bad digits, a stream
    # that decodes past U or short of it -- all re-encoded whole, as the reference does
    for content, U, new in [(b"aa2aa2", 4, b"ab"), (b"aa1", 1, b"a"), (b"aaz", 1, b"q"), (b"aa9", 3, b"a"),
                            (b"abc", 5, b"cc"), (b"a", 3, b"\0"), (b"xx5yy7", 12, b"y"), (b"11", 1, b"1")]:
        assert R.append(content, U, new) == ref_append(content, U, new), (content, U, new)


def test_decompress_n_zero_copy_chunks():
    """Small files go through the mapped buffer in chunks (csrc/rle_dropin.cpp decompress_n_chunk_zc):
    more files than one chunk's launch words (56), inputs past the 256 KiB input region, 16 KiB
    files at the size limit, then one past it, and small files again after it."""
    xs = [O.gen(k % 4, k, 100 + (k * 37) % 4000) for k in range(250)]
    xs += [O.gen(1, 1000 + k, 16384) for k in range(40)] + [O.gen(2, 7, 16385)] + [O.gen(3, 8, 500)] * 5
    ys = [O.encode(x) for x in xs]
    assert R.decompress_n(ys, [len(x) for x in xs]) == xs


def test_decompress_n_matches_per_file_decodes():
    rng = np.random.default_rng(7)
    xs = [O.gen(i % 5, i, int(rng.integers(0, 20000))) for i in range(300)]
    xs += [b"", b"a", bytes(70000), O.gen(1, 9, 200000)]   # empty, tiny, and segmented-path sizes
    ys = [O.encode(x) for x in xs]
    got = R.decompress_n(ys, [len(x) for x in xs])
    bad = [i for i in range(len(xs)) if got[i] != xs[i]]
    assert not bad, bad[:5]


def test_decompress_n_reference_semantics_on_odd_streams():
    # C == 0 with U > 0 (zeros), U shorter than the stream, invalid digits: each equal to RLEdecompress
    streams = [b"", b"aa9aa9", b"aaz", b"ab", b"xx5", b"\0\0\0"]
    us = [7, 4, 3, 6, 5, 2]
    got = R.decompress_n(streams, us)
    for s, u, g in zip(streams, us, got):
        assert g == O.decode(s, u)[0], (s, u)
        assert g == R.decompress(s, u), (s, u)
    assert R.decompress_n([], []) == []
    # U == 0 with a non-empty stream: nothing is decoded (the reference writes into a calloc(0)
    # block); one-wave and segmented stream sizes, with and without an extra region
    big = O.encode(O.gen(1, 3, 40000))
    for s in (b"aa9", b"abc", big):
        assert R.decompress_n([s], [0]) == [b""]
        assert R.decompress(s, 0) == b""
        # with an extra region the reference's unbounded first write (src/rleCompression.c:51)
        # lands in it: the oracle restates that
        assert R.decompress(s, 0, 5) == O.decode(s, 0, 5)[0][:5]
    assert R.decompress_n([b"aa9", big, b"", b"ab"], [0, 0, 0, 1]) == [b"", b"", b"", b"a"]


def test_decompress_n_chunks_past_the_staging_cap():
    # a readN larger than the bounded staging (kStageCap, 32 MiB): consecutive chunks, and a file
    # too large for the staging decoded straight into the caller's buffer
    xs = [O.gen(1 + i % 4, 500 + i, (1 << 20) + 37 * i) for i in range(40)]
    xs.insert(17, bytes(48 << 20))
    xs.append(b"q" * 5)
    ys = [O.encode(x) if i % 7 else R.compress(x) for i, x in enumerate(xs)]
    got = R.decompress_n(ys, [len(x) for x in xs])
    bad = [i for i in range(len(xs)) if got[i] != xs[i]]
    assert not bad, bad[:5]


def test_decompress_n_small_staging_cap_subprocess():
    # the same chunking with a 64 KiB cap (RLE_MI355X_STAGE_CAP), in a fresh process so the cap
    # is read at library init: many small chunks, and mid-size files alone
    import os
    import subprocess
    import sys
    code = (
        "import sys; sys.path[:0] = sys.argv[1:3]\n"
        "import rle_mi355x as R, rle_oracle as O\n"
        "xs = [O.gen(i % 5, 900 + i, (i * 7919) % 90000) for i in range(120)]\n"
        "got = R.decompress_n([O.encode(x) for x in xs], [len(x) for x in xs])\n"
        "assert got == xs, [i for i in range(len(xs)) if got[i] != xs[i]][:5]\n"
        "print('ok')\n")
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    env = dict(os.environ, RLE_MI355X_STAGE_CAP=str(64 << 10))
    r = subprocess.run([sys.executable, "-c", code, os.path.join(root, "c-filestorage-server-and-client_amd"),
                        os.path.join(root, "oracle")], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr[-2000:]


def test_decompress_n_readn_batch_of_fixture_files(dummyfiles):
    from conftest import committed_file_bytes
    xs = [x for x in (committed_file_bytes(e) for e in dummyfiles["files"]) if x is not None]
    ys = [R.compress(x) for x in xs]
    assert R.decompress_n(ys, [len(x) for x in xs]) == xs


def test_fileops_concurrent_threads():
    """The server's worker pool calls these from many threads at once (src/server.c:520-524)."""
    import threading
    errors = []

    def worker(t):
        rng = np.random.default_rng(100 + t)
        content, plain = b"", b""
        for k in range(25):
            new = O.gen(int(rng.integers(0, 5)), t * 100 + k, int(rng.integers(0, 40000)))
            content = R.append(content, len(plain), new)
            plain += new
            if content != O.encode(plain):
                errors.append(("append", t, k))
                return
            if k % 5 == 4:
                xs = [plain[: len(plain) // 3], plain, new]
                if R.decompress_n([O.encode(x) for x in xs], [len(x) for x in xs]) != xs:
                    errors.append(("readN", t, k))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors[:5]


def test_allocation_failure_returns_null_enomem():
    """An allocation the drop-in cannot make returns what the reference's failed calloc gives its
    callers (NULL / -1, errno = ENOMEM; src/filesystemApi.c:598-600, 681-684) instead of aborting
    the server, and the thread's later calls work.  Allocations past 1 MiB are made to fail
    (RLE_MI355X_FAIL_ALLOC_ABOVE, read at library init: a fresh process)."""
    import os
    import subprocess
    import sys
    code = r'''
import ctypes, errno, sys
sys.path[:0] = sys.argv[1:3]
import rle_mi355x as R, rle_oracle as O
L = ctypes.CDLL(R.LIB_PATH, use_errno=True)
L.RLEcompress.restype = ctypes.c_void_p
L.RLEcompress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
L.RLEdecompress.restype = ctypes.c_void_p
L.RLEdecompress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t]
big = O.gen(1, 1, 3 << 20)
c = ctypes.c_size_t(99)
ctypes.set_errno(0)
assert not L.RLEcompress(big, len(big), ctypes.byref(c)) and c.value == 0 and ctypes.get_errno() == errno.ENOMEM
y = O.encode(big)
ctypes.set_errno(0)
assert not L.RLEdecompress(y, len(y), len(big), 0) and ctypes.get_errno() == errno.ENOMEM
xs = [O.gen(2, 7, 2 << 20), O.gen(0, 8, 5000)]
try:
    R.decompress_n([O.encode(x) for x in xs], [len(x) for x in xs])
    raise SystemExit("readN did not fail")
except R.RLEError as e:
    assert "errno %d" % errno.ENOMEM in str(e), e
small = O.gen(3, 9, 40000)
assert R.compress(small) == O.encode(small) and R.decompress(O.encode(small), len(small)) == small
print("ok")
'''
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    # the hook is compiled only into the test build of the library (RLE_TEST_HOOKS)
    testlib = os.path.join(root, "c-filestorage-server-and-client_amd", "build", "librle_mi355x_testhooks.so")
    assert os.path.exists(testlib), "build() makes the test-hook library"
    env = dict(os.environ, RLE_MI355X_FAIL_ALLOC_ABOVE=str(1 << 20), RLE_MI355X_LIB=testlib)
    r = subprocess.run([sys.executable, "-c", code, os.path.join(root, "c-filestorage-server-and-client_amd"),
                        os.path.join(root, "oracle")], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), (r.stdout[-1000:], r.stderr[-2000:])
