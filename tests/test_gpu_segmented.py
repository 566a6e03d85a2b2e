"""GPU parity of the SEGMENTED codec (several waves per buffer: rle_*_batch_device_seg, the path the
drop-in takes for large files) against the oracle, bit-exact.  Segments are 64512 input bytes;
the cases sit on and around segment edges, carry runs and token phases across them (including
'9' runs, whose decode phases never re-synchronise), mix buffer sizes, and feed invalid streams
that must fall back to the exact serial decoder.  The algebra itself is pinned on CPU by
tests/test_seg_model.py."""
import os

import numpy as np
import pytest

import rle_mi355x as R
import rle_oracle as O
from test_gpu_parity import gpu_decode, gpu_encode

pytestmark = pytest.mark.gpu
# segment length of the path under test: 64512 for the four-launch kernels at these batch sizes;
# 7056 (7 tiles) for the resident single-pass kernels (RLE_MI355X_SEG_RES=1, which
# test_resident_single_pass below sets for a second run of this module)
RES = os.environ.get("RLE_MI355X_SEG_RES", "0") == "1"
RES_MODE = os.environ.get("RLE_MI355X_SEG_RES", "0")   # "2": the single pass without the resident segment
S = 7056 if RES else 64512


def _parity(xs):
    ys, st = gpu_encode(xs, seg=True)
    assert (st == 0).all(), st
    for i, x in enumerate(xs):
        ref = O.encode(x)
        assert ys[i] == ref, (i, len(x), len(ys[i]), len(ref))
    dec, st = gpu_decode(ys, [len(x) for x in xs], seg=True)
    for i, x in enumerate(xs):
        assert dec[i] == x, (i, len(x))
    assert ((st & 0xFF) == 0).all(), st
    return ys


def test_segment_edge_sizes():
    xs = []
    for k in (1, 2, 3):
        for d in (-3, -2, -1, 0, 1, 2, 3, 4, 17):
            for kind in range(5):
                xs.append(O.gen(kind, 100 * k + d + 7, k * S + d))
    xs += [b"", b"a", bytes(5), O.gen(1, 1, 1000)]
    _parity(xs)


def test_runs_and_phases_across_segments():
    xs = [bytes(3 * S + 5), b"\xff" * (2 * S + 2), b"9" * (2 * S + 7), b"3" * (S + 3), b"99" * S]
    # a zero run from position 0 (its first tile must not pass for the inside of a run), whole tiles
    # inside runs ending on and off tile edges (the summary's uniform-tile count)
    xs += [bytes(S + 2000) + O.gen(1, 3, S), bytes(2 * S) + b"\x01" + bytes(S)]
    for e in (1007, 1008, 1009, 2016, 2017, 5000):
        xs.append(O.gen(1, e, 3000) + b"q" * (e + S) + O.gen(1, e + 1, S))
    for k in (1, 2, 5, 8, 9, 10, 17, 100):   # a run ending / starting k bytes around a segment edge
        xs.append(b"a" * (S - k) + b"b" * (2 * k + 9) + b"c" * 1000)
        xs.append(O.gen(1, k, S - k) + b"z" * (k + 40) + O.gen(3, k, S))
    # compressed streams whose segment edges fall inside 3-byte tokens at every offset
    for k in range(6):
        xs.append(b"x" * k + b"aaab" * (S // 4 + 10))
    _parity(xs)


@pytest.mark.parametrize("kind", [0, 1, 2, 3, 4])
def test_large_buffers_per_kind(kind):
    xs = [O.gen(kind, 7, 4 << 20), O.gen(kind, 8, (1 << 20) + 12345)]
    _parity(xs)


def test_uniform_segments():
    """Segments without a run boundary are written from the entering run start alone (the write
    pass does not read them again): runs from every phase, ending 0..10 bytes past a segment's end
    (the last token's count), at the buffer's end, and whole zero-filled buffers, for every segment
    length the launcher may pick at these sizes (multiples of 1008)."""
    xs = []
    for m in (4, 7, 16):
        L = m * 1008
        for e in range(11):
            xs.append(O.gen(1, e, 100 + e) + b"z" * (3 * L + e) + O.gen(1, 50 + e, 3000))
            xs.append(b"\x00" * (2 * L + e))
        for ph in range(9):
            xs.append(O.gen(1, 90 + ph, L - ph) + b"\xee" * (2 * L + 17) + b"\xef")
    _parity(xs)


def test_mixed_batch_same_as_one_wave_path():
    rng = np.random.default_rng(11)
    xs = []
    for i in range(96):
        U = int(2 ** rng.uniform(12, 20)) + int(rng.integers(0, 64))
        xs.append(O.gen(i % 4, i, U))
    ys_seg = _parity(xs)
    ys_one, st = gpu_encode(xs)
    assert ys_one == ys_seg and (st == 0).all()


def test_invalid_streams_take_the_serial_path():
    good = O.encode(O.gen(2, 3, 3 * S))
    bad_digit = bytearray(good)
    pos = 2 * S + 100
    while not (bad_digit[pos] == bad_digit[pos + 1]):
        pos += 1
    bad_digit[pos + 2] = ord(":")            # count digit outside '1'..'9'
    streams = [bytes(bad_digit), good, good[:-1] + b"q", b"aa9" * 40000, b"\x07" * (S + 10) + b"\x00"]
    us = [3 * S, 3 * S, 3 * S, 10 * S, 2 * S]
    caps = [u + 64 for u in us]
    dec, st = gpu_decode(streams, us, caps, poison=False, seg=True)
    for i, (y, U, cap) in enumerate(zip(streams, us, caps)):
        ref, _ = O.decode(y, U, cap)
        assert dec[i] == ref, i
    assert st[0] & R.RLE_STATUS_SERIAL


def test_one_buffer_launches():
    """A segmented launch of ONE buffer takes its segments from its length, without the plan and map
    launches (rle_segmented.hip RLE_SEG_ONE): every kind at and around segment edges, the empty and
    one-byte buffers, a stream that declines to the serial path and one that decodes short."""
    cases = [b"", b"a", bytes(3), O.gen(1, 3, 1000)]
    for k in (1, 2, 4):
        for d in (-2, 0, 1, 3):
            for kind in range(5):
                cases.append(O.gen(kind, 10 * k + d + kind, k * S + d))
    for x in cases:
        _parity([x])
    good = O.encode(O.gen(2, 5, 2 * S))
    bad = bytearray(good)
    pos = S + 50
    while bad[pos] != bad[pos + 1]:
        pos += 1
    bad[pos + 2] = ord(":")
    for y, U in ((bytes(bad), 2 * S), (good, 2 * S + 9)):
        dec, st = gpu_decode([y], [U], [U + 16], poison=False, seg=True)
        ref, _ = O.decode(y, U, U + 16)
        assert dec[0] == ref


def test_dropin_large_files_roundtrip():
    for x in (O.gen(1, 5, 3 << 20), bytes(2 << 20), O.gen(3, 6, (1 << 20) + 1)):
        y = R.compress(x)
        assert y == O.encode(x)
        assert R.decompress(y, len(x), 5) == x + bytes(5)


def test_dropin_very_large_file():
    """A 192 MiB file through the drop-in: the runtime's direct copies, the segmented kernels with
    thousands of segments, and the reference's result byte for byte."""
    x = O.gen(2, 77, 192 << 20)
    y = R.compress(x)
    assert y == O.encode(x)
    assert R.decompress(y, len(x)) == x


_FUSED_CODE = r'''
import sys
sys.path[:0] = sys.argv[1:4]
import rle_oracle as O
from test_gpu_segmented import S
from test_gpu_parity import gpu_encode
xs = [bytes(3 * S + 5), O.gen(1, 1, 5 * S + 7), O.gen(2, 2, 2 * S), b"q" * (4 * S + 1), b"", b"a"]
xs += [O.gen(k % 5, 40 + k, (k + 1) * 7000) for k in range(40)]
xs.append(O.gen(3, 9, 64 << 20))   # one buffer of thousands of segments (the longest look-back)
ys, st = gpu_encode(xs, seg=True)
assert (st == 0).all(), st
for i, x in enumerate(xs):
    assert ys[i] == O.encode(x), (i, len(x))
print("ok")
'''


def _variants_lib(root):
    """The fused and resident kernels are measured slower than the default and live only in the test
    build (RLE_VARIANTS, c-filestorage-server-and-client_amd/Makefile), not in the product library."""
    p = os.path.join(root, "c-filestorage-server-and-client_amd", "build", "librle_mi355x_testhooks.so")
    assert os.path.exists(p), "build() makes the test library"
    return p


def test_fused_single_pass_encode():
    """The fused single-pass segmented encode (RLE_MI355X_SEG_FUSED=1, read at load: a fresh
    process): ticket-ordered segments, write-through summaries and inclusive states, the decoupled
    look-back, against the oracle -- including a 64 MiB buffer whose segments look back thousands
    of places."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    env = dict(os.environ, RLE_MI355X_SEG_FUSED="1", RLE_MI355X_LIB=_variants_lib(root))
    r = subprocess.run([sys.executable, "-c", _FUSED_CODE, os.path.join(root, "c-filestorage-server-and-client_amd"),
                        os.path.join(root, "oracle"), here], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "ok" in r.stdout, (r.stdout[-1500:], r.stderr[-3000:])


@pytest.mark.parametrize("mode", ["1", "2"])
def test_resident_single_pass(mode):
    """The single-pass segmented kernels (read at load: a fresh process): RLE_MI355X_SEG_RES=1, the
    resident form (encode and decode; the segment edges at its segment length), and =2, the decode
    without the resident segment (round 5: its write walk re-reads the segment): this whole module
    again, plus the drop-in's large files, against the oracle."""
    if RES_MODE != "0":
        pytest.skip("already a single-pass run")
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, RLE_MI355X_SEG_RES=mode, RLE_MI355X_LIB=_variants_lib(os.path.dirname(here)))
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-m", "gpu", "-p", "no:cacheprovider",
                        os.path.join(here, "test_gpu_segmented.py"), "-k", "not fused and not resident"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
