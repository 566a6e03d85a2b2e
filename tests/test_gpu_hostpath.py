"""GPU tests of the drop-in's host path (BASELINE configs[4]).

* The registered large calls (the default past the zero-copy reach) and every staging mode a call
  falls back to (RLE_MI355X_STAGING = direct / pinned / pipe, read at library init: a fresh process
  each) give the oracle's bytes for RLEcompress / RLEdecompress across the size thresholds
  (zero-copy small calls, pinned one-trip, segmented, >= 256 KiB), for RLEappend and for
  RLEdecompressN with a file past the staging cap; registered calls from eight threads on buffers
  that share pages, on one shared stream, on overlapping ranges and on read-only pages.
* Concurrent small calls from many threads (the server's worker pool, src/server.c:520-524) stay
  bit-exact, on per-thread streams (the default) and combined into shared launches
  (RLE_MI355X_COALESCE=1): each thread's streams against the oracle, and the C call-rate tool's
  round trips.
"""
import json
import os
import subprocess
import sys
import threading

import pytest

import rle_mi355x as R
import rle_oracle as O

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

_STAGING_CODE = r'''
import sys
sys.path[:0] = sys.argv[1:3]
import rle_mi355x as R, rle_oracle as O
sizes = [1, 13, 4096, 40000, 70000, 200000, 300000, 2 << 20, 5 << 20]
for i, U in enumerate(sizes):
    for kind in (0, 1, 2, 3):
        x = O.gen(kind, 1000 * i + kind, U)
        y = O.encode(x)
        assert R.compress(x) == y, (U, kind)
        assert R.decompress(y, U) == x, (U, kind)
        assert R.decompress(y, U, 777) == x + bytes(777), (U, kind)
# the write path (src/filesystemApi.c:766-775) fused
for U, A in ((4096, 4096), (300000, 70000), (3 << 20, 1 << 20)):
    old = O.gen(2, U, U)
    new = O.gen(3, A, A)
    assert R.append(O.encode(old), U, new) == O.encode(old + new), (U, A)
# readNFiles: small files, one past the 64 KiB staging cap set below, an empty one
xs = [O.gen(k % 4, 50 + k, s) for k, s in enumerate([4096, 300000, 1000, 0, 70000, 2 << 20])]
assert R.decompress_n([O.encode(x) for x in xs], [len(x) for x in xs]) == xs
print("ok", R.dropin_stats())
'''


# call coalescing and pipelined staging are measured slower than the defaults and live only in the
# test build (RLE_VARIANTS, c-filestorage-server-and-client_amd/Makefile), not in the product library
VARIANTS_LIB = os.path.join(ROOT, "c-filestorage-server-and-client_amd", "build", "librle_mi355x_testhooks.so")


@pytest.mark.parametrize("mode", ["registered", "direct", "pinned", "pipe"])
def test_staging_modes_bit_exact(mode):
    # "registered" is the default (large calls on the caller's registered memory); the staging modes
    # are what a call falls back to, so they run with the registered path off
    env = dict(os.environ, RLE_MI355X_STAGE_CAP=str(1 << 20))
    if mode != "registered":
        env.update(RLE_MI355X_STAGING=mode, RLE_MI355X_REG_MIN="0")
    if mode == "pipe":
        env["RLE_MI355X_LIB"] = VARIANTS_LIB
    r = subprocess.run([sys.executable, "-c", _STAGING_CODE, os.path.join(ROOT, "c-filestorage-server-and-client_amd"),
                        os.path.join(ROOT, "oracle")], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "ok" in r.stdout, (r.stdout[-1500:], r.stderr[-3000:])


_REG_CODE = r'''
import sys, ctypes, mmap, os, tempfile, threading
sys.path[:0] = sys.argv[1:3]
import numpy as np
import rle_mi355x as R, rle_oracle as O
L = ctypes.CDLL(R.lib()._name)
sz = ctypes.c_size_t
L.RLEcompress.restype = ctypes.c_void_p
L.RLEcompress.argtypes = [ctypes.c_void_p, sz, ctypes.POINTER(sz)]
L.RLEdecompress.restype = ctypes.c_void_p
L.RLEdecompress.argtypes = [ctypes.c_void_p, sz, sz, sz]
free = R._libc.free

def comp(addr, U):
    c = sz(0)
    p = L.RLEcompress(addr, U, ctypes.byref(c))
    assert p
    y = ctypes.string_at(p, c.value + 16)
    free(p)
    assert y[c.value:] == bytes(16)
    return y[:c.value]

def decomp(addr, C, U, E):
    p = L.RLEdecompress(addr, C, U, E)
    assert p
    y = ctypes.string_at(p, U + E)
    free(p)
    return y

R.dropin_stats(reset=True)
# neighbouring slices of one buffer (their pages shared), odd sizes and offsets, kinds mixed
sizes = [70001, 100003, 262145, 300007, 1048579, 777777, 2 << 20, 130001]
offs = [16 + sum(sizes[:i]) + 3 * i for i in range(len(sizes))]
big = np.zeros(offs[-1] + sizes[-1] + 64, dtype=np.uint8)
xs = [O.gen(i % 4, 300 + i, U) for i, U in enumerate(sizes)]
for o, x in zip(offs, xs):
    big[o:o + len(x)] = np.frombuffer(x, dtype=np.uint8)
ys = [O.encode(x) for x in xs]
yoffs = [8 + sum(len(y) for y in ys[:i]) + 5 * i for i in range(len(ys))]
ybig = np.zeros(yoffs[-1] + len(ys[-1]) + 64, dtype=np.uint8)
for o, y in zip(yoffs, ys):
    ybig[o:o + len(y)] = np.frombuffer(y, dtype=np.uint8)
base, ybase = big.ctypes.data, ybig.ctypes.data
errors = []
# alone: registered
assert comp(base + offs[4], sizes[4]) == ys[4]
assert decomp(ybase + yoffs[4], len(ys[4]), sizes[4], 100) == xs[4] + bytes(100)
assert R.dropin_stats()["calls_registered"] == 2, R.dropin_stats()

def work(t):
    try:
        for rep in range(3):
            for k in range(len(sizes)):
                i = (k + t) % len(sizes)
                if comp(base + offs[i], sizes[i]) != ys[i]:
                    errors.append(("c", t, i))
                E = 0 if (t + rep) % 2 else 4097
                if decomp(ybase + yoffs[i], len(ys[i]), sizes[i], E) != xs[i] + bytes(E):
                    errors.append(("d", t, i))
                # every thread also reads the same stored stream (one shared registration)
                if decomp(ybase + yoffs[6], len(ys[6]), sizes[6], 0) != xs[6]:
                    errors.append(("s", t))
    except Exception as e:   # noqa: BLE001
        errors.append(repr(e))

# beside them, the readN and append paths on the same stored stream (a file past the staging cap
# set for this process: its bytes go straight from / to caller memory, or through the staging in
# chunks while another call holds a registration)
def other(t):
    try:
        for rep in range(4):
            y6 = ctypes.string_at(ybase + yoffs[6], len(ys[6]))
            if R.decompress_n([y6, ys[1]], [sizes[6], sizes[1]]) != [xs[6], xs[1]]:
                errors.append(("n", t))
            if R.append(y6, sizes[6], xs[3]) != O.encode(xs[6] + xs[3]):
                errors.append(("a", t))
    except Exception as e:   # noqa: BLE001
        errors.append(repr(e))

th = [threading.Thread(target=work, args=(t,)) for t in range(8)] + [threading.Thread(target=other, args=(9,))]
for t in th: t.start()
for t in th: t.join()
assert not errors, errors[:10]
# overlapping ranges of one buffer from two threads
x2 = O.gen(2, 99, 3 << 20)
b2 = np.frombuffer(x2, dtype=np.uint8).copy()
refs = {(0, 2 << 20): O.encode(x2[:2 << 20]), (1 << 20, 2 << 20): O.encode(x2[1 << 20:3 << 20])}
def ov(o):
    for _ in range(6):
        if comp(b2.ctypes.data + o, 2 << 20) != refs[(o, 2 << 20)]:
            errors.append(("ov", o))
th = [threading.Thread(target=ov, args=(o,)) for o in (0, 1 << 20)]
for t in th: t.start()
for t in th: t.join()
assert not errors, errors[:10]
# read-only pages: a file mapped read-only
x3 = O.gen(3, 5, 1500000)
with tempfile.NamedTemporaryFile(delete=False) as f:
    f.write(x3)
with open(f.name, "rb") as fh:
    mm = mmap.mmap(fh.fileno(), 0, access=mmap.ACCESS_READ)
    a = np.frombuffer(mm, dtype=np.uint8)
    assert comp(a.ctypes.data, len(x3)) == O.encode(x3)
    del a
    mm.close()
os.unlink(f.name)
st = R.dropin_stats()
assert st["calls_registered"] > 0, st
print("ok", st)
'''


def test_registered_large_calls_concurrent_bit_exact():
    """Large calls on the caller's registered memory (the default past 256 KiB, when a call is the
    only large call in flight; csrc/rle_dropin.cpp LargeCall): alone; eight threads on neighbouring
    slices of one buffer, whose pages they share, and on one stored stream that all of them read
    while a ninth runs readN and append on it (past a 1 MiB staging cap); two threads on overlapping
    ranges; a read-only mapped file; all bit-exact against the oracle."""
    r = subprocess.run([sys.executable, "-c", _REG_CODE, os.path.join(ROOT, "c-filestorage-server-and-client_amd"),
                        os.path.join(ROOT, "oracle")],
                       env=dict(os.environ, RLE_MI355X_STAGE_CAP=str(1 << 20), RLE_MI355X_REG_MIN=str((256 << 10) + 1),
                                RLE_MI355X_REG_QUIET_US="2000"),
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "ok" in r.stdout, (r.stdout[-1500:], r.stderr[-3000:])


def test_registered_calls_on_streams_the_encoder_never_writes():
    """Registered decompress (past 256 KiB) of streams that are not encoder output, with an extra
    region: the exact serial decode may write into the E region, which then travels too
    (decompress_registered); streams that decode short of U, past U, and exactly to it."""
    rng = __import__("random").Random(5)
    cases = []
    for C in (300001, 700000, 1 << 20):
        s = rng.randbytes(C)   # random bytes read as a stream
        for U, E in ((C // 2, 4096), (C, 100), (2 * C, 333), (C + 7, 0)):
            cases.append((s, U, E))
    # an encoder stream with a digit run rewritten (decodes past U), and a valid one cut short
    y = O.encode(O.gen(3, 11, 900000))
    cases.append((y[:len(y) // 2] + b"779" * 1000 + y[len(y) // 2:], 900000, 5000))
    cases.append((y, 800000, 12345))
    for s, U, E in cases:
        got = R.decompress(s, U, E)
        ref, _ = O.decode(s, U, U + E)
        assert got == ref, (len(s), U, E)


_COALESCE_CODE = r'''
import sys, threading
sys.path[:0] = sys.argv[1:3]
import rle_mi355x as R, rle_oracle as O
R.dropin_stats(reset=True)
errors = []
inputs = [[O.gen(k % 4, 7000 + 100 * t + k, 4096 + 9000 * (k % 5)) for k in range(40)] for t in range(16)]
refs = [[O.encode(x) for x in xs] for xs in inputs]

def work(t):
    try:
        for x, y in zip(inputs[t], refs[t]):
            if R.compress(x) != y:
                errors.append(("enc", t, len(x)))
            if R.decompress(y, len(x), 3) != x + bytes(3):
                errors.append(("dec", t, len(x)))
    except Exception as e:   # surfaced below
        errors.append(repr(e))

th = [threading.Thread(target=work, args=(t,)) for t in range(16)]
for x in th:
    x.start()
for x in th:
    x.join()
assert not errors, errors[:5]
st = R.dropin_stats()
# every compress is a zero-copy call (U < 48 KiB); decompress is from C < 32 KiB
small = 16 * 40 + sum(len(y) < (32 << 10) for ys in refs for y in ys)
assert st["calls_coalesced"] == small
assert 0 < st["launches_coalesced"] <= st["calls_coalesced"]
print("ok", st)
'''


def test_concurrent_small_calls_coalesced_bit_exact():
    """With call coalescing on (RLE_MI355X_COALESCE=1, read at init: a fresh process): 16 Python
    threads, each 40 round trips of its own 4 KiB - 40 KiB buffers through the drop-in, every stream
    against the oracle; the library counts every small call as combined."""
    # (no background start-up: its warm-up calls would be combined too, after the counters' reset)
    # (and the one-wave zero-copy range only: the count below is of calls under 48 / 32 KiB)
    # (coalescing combines zero-copy calls: RLE_MI355X_SMALL from the caller's environment is reset)
    env = dict(os.environ, RLE_MI355X_COALESCE="1", RLE_MI355X_LIB=VARIANTS_LIB, RLE_MI355X_PREINIT="0",
               RLE_MI355X_ZC_SEG="0", RLE_MI355X_SMALL="zerocopy")
    r = subprocess.run([sys.executable, "-c", _COALESCE_CODE, os.path.join(ROOT, "c-filestorage-server-and-client_amd"),
                        os.path.join(ROOT, "oracle")], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "ok" in r.stdout, (r.stdout[-1500:], r.stderr[-3000:])


def test_concurrent_small_calls_per_thread_streams_bit_exact():
    """The default (one stream per calling thread, no combining): 16 threads of 4 KiB - 40 KiB round
    trips against the oracle, and no call was combined."""
    R.dropin_stats(reset=True)
    errors = []
    inputs = [[O.gen(k % 4, 9000 + 100 * t + k, 4096 + 9000 * (k % 5)) for k in range(20)] for t in range(16)]

    def work(t):
        try:
            for x in inputs[t]:
                y = O.encode(x)
                if R.compress(x) != y or R.decompress(y, len(x)) != x:
                    errors.append((t, len(x)))
        except Exception as e:
            errors.append(repr(e))

    th = [threading.Thread(target=work, args=(t,)) for t in range(16)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors[:5]
    assert R.dropin_stats()["calls_coalesced"] == 0


@pytest.mark.parametrize("coalesce", ["0", "1"])
def test_callrate_tool_round_trips(coalesce):
    """The C call-rate tool (8 threads x 4 KiB, 1 s) on the product library: every round trip exact;
    RLE_MI355X_COALESCE=1 is not read by the product build (no call is combined)."""
    exe = os.path.join(ROOT, "tools", "callrate")
    assert os.path.exists(exe), "build() compiles tools/callrate"
    r = subprocess.run([exe, "8", "4096", "1"], capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, RLE_MI355X_COALESCE=coalesce))
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["bad"] == 0 and out["calls"] > 0
    assert out["calls_coalesced"] == 0


_POLL_CODE = r'''
import sys, threading
sys.path[:0] = sys.argv[1:3]
import numpy as np
import rle_mi355x as R, rle_oracle as O
rng = np.random.default_rng(5)
errors = []
# one thread: consecutive calls of different content through the same mapped buffer, so output
# left from an earlier call (a flag seen before the output) would show
for k in range(600):
    U = int(rng.integers(0, 16385))
    x = O.gen(k % 5, 40000 + k, U)
    y = O.encode(x)
    if R.compress(x) != y:
        errors.append(("enc", k, U))
    E = int(rng.integers(0, 40))
    if R.decompress(y, U, E) != x + bytes(E):
        errors.append(("dec", k, U, E))
    if k % 7 == 0:   # streams the encoder never emits: serial decode, the extra region filled
        s = b"aa:" + y[:3000]
        if R.decompress(s, U, 64) != O.decode(s, U, U + 64)[0]:
            errors.append(("serial", k, U))

# 32-64 KiB calls (the zero-copy segmented form's upper range with RLE_MI355X_ZC_SEG; the copying
# large-call form otherwise), exactly 64 KiB, and decodes with a large extra region
for k in range(40):
    U = 65536 if k % 10 == 9 else 32768 + (k * 997) % 32768
    x = O.gen(k % 5, 60000 + k, U)
    y = O.encode(x)
    if R.compress(x) != y:
        errors.append(("enc-mid", k, U))
    E = 50000 if k % 3 == 0 else 0
    if R.decompress(y, U, E) != x + bytes(E):
        errors.append(("dec-mid", k, U, E))

# 64-400 KiB calls: past the cooperative kernels, the zero-copy segmented form up to its 256 KiB of
# input (and 384 KiB of output), the copying form past it; sizes at both reaches
for k, U in enumerate([65537, 80640, 80641, 98304, 131072, 200000, 262143, 262144, 262145, 300000, 409600]):
    x = O.gen(k % 5, 70000 + k, U)
    y = O.encode(x)
    if R.compress(x) != y:
        errors.append(("enc-big", k, U))
    E = 393216 - U if k % 2 == 0 and U < 393216 else 0   # the output region's reach, exactly
    got = R.decompress(y, U, E)
    if got != x + bytes(E):   # (where and how: the first differing byte, the path's counters)
        want = x + bytes(E)
        i = next(j for j in range(len(want)) if j >= len(got) or got[j] != want[j])
        errors.append(("dec-big", k, U, E, len(y), i, got[i:i + 8].hex(), want[i:i + 8].hex(), R.dropin_stats()))

def work(t):
    try:
        for k in range(150):
            U = 1 + (k * 977 + t * 131) % 12000
            x = O.gen((k + t) % 5, 90000 + 1000 * t + k, U)
            y = O.encode(x)
            if R.compress(x) != y or R.decompress(y, U) != x:
                errors.append(("thread", t, k, U))
    except Exception as e:
        errors.append(repr(e))

th = [threading.Thread(target=work, args=(t,)) for t in range(8)]
for x in th:
    x.start()
for x in th:
    x.join()
assert not errors, errors[:5]
print("ok")
'''


@pytest.mark.parametrize("poll,service,zcseg,one", [("1", "0", "0", "1"), ("0", "0", "0", "1"), ("1", "1", "0", "1"),
                                                    ("1", "0", "8192", "1"), ("1", "0", "0", "0")])
def test_polled_small_calls_bit_exact(poll, service, zcseg, one):
    """The zero-copy small calls' completion: polling the status word the kernel stores behind a
    system-scope release (RLE_MI355X_POLL=1, the default) or hipStreamSynchronize (=0), or the
    resident service (RLE_MI355X_SERVICE=1: no launch per call, csrc/rle_service.h; built into the
    RLE_VARIANTS test library only since round 5, so that case loads it).  600
    consecutive calls of 0-16 KiB (cooperative and one-wave kernels), decodes with an extra region,
    serial-path streams, then 8 threads x 150 round trips, all against the oracle.  zcseg: calls
    from that many bytes run the segmented kernels on the mapped buffer (RLE_MI355X_ZC_SEG).  one:
    the cooperative kernels take a single call's sizes as arguments (RLE_MI355X_COOP_ONE=1, the
    default since round 6) or read them from the mapped launch words (=0, the batched entry points)."""
    env = dict(os.environ, RLE_MI355X_POLL=poll, RLE_MI355X_SERVICE=service, RLE_MI355X_ZC_SEG=zcseg,
               RLE_MI355X_COOP_ONE=one)
    if service == "1":
        env["RLE_MI355X_LIB"] = VARIANTS_LIB
    r = subprocess.run([sys.executable, "-c", _POLL_CODE, os.path.join(ROOT, "c-filestorage-server-and-client_amd"),
                        os.path.join(ROOT, "oracle")], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "ok" in r.stdout, (r.stdout[-1500:], r.stderr[-3000:])


_SERVICE_CODE = r"""
import sys, threading, time
sys.path[:0] = sys.argv[1:3]
import rle_mi355x as R, rle_oracle as O
errors = []
# calls spaced past the service's idle time (1 ms): every call finds it gone and relaunches it
for k in range(20):
    x = O.gen(k % 5, 500 + k, 1000 + 700 * k)
    y = O.encode(x)
    if R.compress(x) != y or R.decompress(y, len(x)) != x:
        errors.append(("gap", k))
    time.sleep(0.003)
# many threads at once: one resident service workgroup each
def work(t):
    try:
        for k in range(6):
            U = 1 + (k * 3001 + t * 17) % 20000
            x = O.gen((k + t) % 5, 70000 + 100 * t + k, U)
            y = O.encode(x)
            if R.compress(x) != y or R.decompress(y, U, 5) != x + bytes(5):
                errors.append(("thread", t, k))
    except Exception as e:
        errors.append(repr(e))
th = [threading.Thread(target=work, args=(t,)) for t in range(72)]
for x in th:
    x.start()
for x in th:
    x.join()
assert not errors, errors[:5]
print("ok")
"""


def test_service_relaunch_and_overflow_bit_exact():
    """The resident service (RLE_MI355X_SERVICE=1) across its own idle exits (calls 3 ms apart: a
    relaunch each) and with 72 threads at once (72 resident workgroups, one per thread context),
    every stream against the oracle; the process then exits with every service stopped.  (The
    service is built into the RLE_VARIANTS test library only.)"""
    env = dict(os.environ, RLE_MI355X_SERVICE="1", RLE_MI355X_LIB=VARIANTS_LIB)
    r = subprocess.run([sys.executable, "-c", _SERVICE_CODE, os.path.join(ROOT, "c-filestorage-server-and-client_amd"),
                        os.path.join(ROOT, "oracle")], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "ok" in r.stdout, (r.stdout[-1500:], r.stderr[-3000:])
