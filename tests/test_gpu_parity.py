"""GPU parity tests: the HIP codec (through librle_mi355x.so's C ABI) against the oracle, the
golden vectors of the compiled reference and the reference fixture pins.  Bit-exact everywhere.

Slots are poisoned before each launch so a write past C (encode) or past U (decode) shows up."""
import hashlib
import threading

import numpy as np
import pytest
import torch

import rle_mi355x as R
import rle_oracle as O
from conftest import committed_file_bytes

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
POISON = 0xA5


def sha(b):
    return hashlib.sha256(b).hexdigest()


def _i64(vals):
    return torch.tensor(np.asarray(vals, dtype=np.int64), device=DEV)


def gpu_encode(bufs, seg=False, max_len=None, flags=0, one_pass=False):
    """Encode a list of byte strings in ONE batched launch (seg: the segmented multi-wave form;
    max_len: the sized entry point with that hint, which picks the cooperative kernels for small
    buffers; one_pass: a workgroup per buffer in rounds, rle_encode_stream_launch); returns
    (outputs, status)."""
    n = len(bufs)
    sizes = [len(b) for b in bufs]
    in_offs, in_total = R.layout(sizes)
    host = np.zeros(in_total, np.uint8)
    for b, o in zip(bufs, in_offs):
        host[o:o + len(b)] = np.frombuffer(b, np.uint8)
    out_offs, out_total = R.compressed_slots(sizes)
    d_in = torch.from_numpy(host).to(DEV)
    d_out = torch.full((out_total + 16,), POISON, dtype=torch.uint8, device=DEV)
    out_len = torch.zeros(n, dtype=torch.int64, device=DEV)
    status = torch.full((n,), 0x7777, dtype=torch.int32, device=DEV)
    if one_pass:
        R.encode_batch_stream(d_in, _i64(in_offs), _i64(sizes), d_out, _i64(out_offs), out_len, status, flags=flags)
    elif max_len is not None:
        R.encode_batch(d_in, _i64(in_offs), _i64(sizes), d_out, _i64(out_offs), out_len, status, max_len=max_len,
                       flags=flags)
    else:
        (R.encode_batch_seg if seg else R.encode_batch)(d_in, _i64(in_offs), _i64(sizes), d_out, _i64(out_offs),
                                                        out_len, status)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    lens = out_len.cpu().numpy()
    res = []
    for i in range(n):
        o, c = out_offs[i], int(lens[i])
        res.append(out[o:o + c].tobytes())
        cap_end = out_offs[i + 1] if i + 1 < n else out_total
        assert (out[o + c:cap_end] == POISON).all(), f"encode wrote past C in buffer {i}"
    return res, status.cpu().numpy()


def gpu_decode(streams, usizes, caps=None, poison=True, seg=False, max_in_len=None, max_out_len=None, flags=0):
    n = len(streams)
    caps = caps if caps is not None else list(usizes)
    in_offs, in_total = R.layout([len(s) for s in streams])
    host = np.zeros(in_total, np.uint8)
    for s, o in zip(streams, in_offs):
        host[o:o + len(s)] = np.frombuffer(s, np.uint8)
    out_offs, out_total = R.layout(caps)
    d_in = torch.from_numpy(host).to(DEV)
    d_out = torch.full((out_total + 16,), POISON if poison else 0, dtype=torch.uint8, device=DEV)
    status = torch.full((n,), 0x7777, dtype=torch.int32, device=DEV)
    if max_in_len is not None:
        R.decode_batch(d_in, _i64(in_offs), _i64([len(s) for s in streams]), d_out, _i64(out_offs), _i64(usizes),
                       _i64(caps), status, max_in_len=max_in_len, max_out_len=max_out_len, flags=flags)
    else:
        (R.decode_batch_seg if seg else R.decode_batch)(d_in, _i64(in_offs), _i64([len(s) for s in streams]), d_out,
                                                        _i64(out_offs), _i64(usizes), _i64(caps), status)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    res = [out[o:o + c].tobytes() for o, c in zip(out_offs, caps)]
    return res, status.cpu().numpy()


def test_selftest_dpp_primitives():
    assert R.selftest() == 0


def test_golden_vectors_encode_decode(vectors):
    cases = [v for g in ("kat", "edge", "ladder", "fuzz") for v in vectors[g]]
    xs = [bytes.fromhex(v["in"]) for v in cases]
    ys = [bytes.fromhex(v["out"]) for v in cases]
    got, st = gpu_encode(xs)
    assert (st == 0).all()
    bad = [i for i in range(len(xs)) if got[i] != ys[i]]
    assert not bad, (len(bad), cases[bad[0]], got[bad[0]].hex())
    dec, st = gpu_decode(ys, [len(x) for x in xs])
    bad = [i for i in range(len(xs)) if dec[i] != xs[i]]
    assert not bad, (len(bad), cases[bad[0]], dec[bad[0]].hex())
    assert ((st & 0xFF) == 0).all()


def test_invalid_streams_match_reference(vectors):
    cases = vectors["invalid_decode"]
    streams = [bytes.fromhex(v["in"]) for v in cases]
    us = [v["U"] for v in cases]
    caps = [v["U"] + v["E"] for v in cases]
    dec, st = gpu_decode(streams, us, caps, poison=False)
    bad = [i for i in range(len(cases)) if dec[i] != bytes.fromhex(cases[i]["out"])]
    assert not bad, (len(bad), cases[bad[0]], dec[bad[0]].hex())
    assert ((st & 0xFF) == 0).all()


def test_decode_overflow_status():
    dec, st = gpu_decode([b"aa9" * 3, b"aa9"], [2, 9], [2, 9])
    assert st[0] & R.RLE_STATUS_OVERFLOW and dec[0] == b"aa"
    assert st[1] == 0 and dec[1] == b"a" * 9


def test_synthetic_pins_and_device_generator(vectors):
    cases = [v for v in vectors["synthetic"]]
    n = len(cases)
    sizes = [v["U"] for v in cases]
    offs, total = R.layout(sizes)
    d = torch.zeros(total, dtype=torch.uint8, device=DEV)
    R.gen_synthetic(d, _i64(offs), _i64(sizes), torch.tensor([v["kind"] for v in cases], dtype=torch.int32,
                                                              device=DEV), _i64([v["index"] for v in cases]))
    torch.cuda.synchronize()
    h = d.cpu().numpy()
    xs = [h[o:o + s].tobytes() for o, s in zip(offs, sizes)]
    for x, v in zip(xs, cases):
        assert sha(x) == v["sha_in"], v
    got, st = gpu_encode(xs)
    for y, v in zip(got, cases):
        assert len(y) == v["C"] and sha(y) == v["sha_out"], v
    dec, st = gpu_decode(got, sizes)
    assert all(a == b for a, b in zip(dec, xs)) and ((st & 0xFF) == 0).all()


def _oracle_parity(xs):
    ys, st = gpu_encode(xs)
    assert (st == 0).all()
    for i, x in enumerate(xs):
        ref = O.encode(x)
        assert ys[i] == ref, (i, len(x), len(ys[i]), len(ref))
    dec, st = gpu_decode(ys, [len(x) for x in xs])
    for i, x in enumerate(xs):
        assert dec[i] == x, (i, len(x))
    assert ((st & 0xFF) == 0).all()
    return ys


def test_config1_4096x4k_roundtrip():
    # BASELINE configs[1]: 4096 synthetic 4 KiB buffers (random / zero), bit-exact vs CPU
    xs = [O.gen(1 if i % 2 == 0 else 0, i, 4096) for i in range(4096)]
    _oracle_parity(xs)


def test_ragged_sizes_and_tile_edges():
    sizes = list(range(0, 130)) + [1023, 1024, 1025, 1026, 1039, 2047, 2048, 2049, 3071, 3072, 4095, 4096, 4097,
                                   8191, 8193, 16383, 16385]
    xs = []
    for k in range(5):
        for i, s in enumerate(sizes):
            xs.append(O.gen(k, 1000 + i, s))
    rng = np.random.default_rng(3)
    for i in range(300):  # digit-heavy and repeat-heavy content around tile edges
        s = int(rng.integers(900, 2300))
        alpha = np.frombuffer(rng.choice([b"a0123456789", b"\0\x01", b"33", b"ab"]), np.uint8)
        runs = rng.integers(1, 22, size=s)
        vals = rng.choice(alpha, size=s)
        xs.append(np.repeat(vals, runs)[:s].tobytes())
    _oracle_parity(xs)


def test_encode_tile_forms_at_their_edges():
    """Both encode tile forms (csrc/rle_device.h enc_tile: 1024-byte tiles for buffers up to 16 KiB
    where they save a tile, 1008-byte overlapped tiles otherwise) at sizes around every multiple
    of 1008 and 1024 up to 17 tiles, with runs that end, or cross a tile boundary, 1..10 bytes
    before or after it (the lookahead bits of lane 63, the 9-byte token cut, digits '1'..'9')."""
    xs = []
    for k in range(1, 18):
        for base in (1008 * k, 1024 * k):
            for d in (-17, -9, -2, -1, 0, 1, 2, 8, 9, 16, 17):
                n = base + d
                xs.append(O.gen(k % 5, n, n))
                for r in (1, 2, 3, 8, 9, 10):
                    for side in (-1, 1):
                        edge = 1024 * (k - 1) + (1024 if side > 0 else 1008)
                        x = bytearray(O.gen(1, 31 * n + r, n))
                        lo, hi = max(0, edge - r), min(n, edge + r * (side > 0))
                        x[lo:hi] = b"7" * (hi - lo)
                        xs.append(bytes(x))
    _oracle_parity(xs)


def test_long_runs_across_tiles():
    xs = [bytes(1 << 20), b"\xff" * 100000, b"a" * 9 * 1024, b"a" * (9 * 1024 + 1), b"\0" * 1023 + b"a" * 3000,
          O.gen(3, 5, 1 << 20), O.gen(4, 5, 300001), O.gen(2, 6, 777777)]
    _oracle_parity(xs)


@pytest.mark.parametrize("kind", [0, 1, 2, 3, 4])
def test_64k_batch_per_kind(kind):
    xs = [O.gen(kind, i, 65536) for i in range(512)]
    _oracle_parity(xs)


def test_mixed_sizes_batch():
    xs = []
    for i in range(160):
        s = np.random.default_rng(i).integers(0, 9)
        U = (1 << (12 + int(s))) + (int(np.random.default_rng(i + 99).integers(0, 4096)) if i % 2 else 0)
        xs.append(O.gen(i % 4, i, U))
    _oracle_parity(xs)


def test_reference_fixture_files(dummyfiles):
    xs, pins = [], []
    for e in dummyfiles["files"]:
        x = committed_file_bytes(e)
        if x is not None:
            xs.append(x)
            pins.append(e)
    ys, st = gpu_encode(xs)
    for y, e in zip(ys, pins):
        assert len(y) == e["C"] and sha(y) == e["sha_out"], e["path"]
    dec, st = gpu_decode(ys, [len(x) for x in xs])
    assert all(a == b for a, b in zip(dec, xs))


def test_dropin_compress_decompress(dummyfiles):
    assert R.compress(b"aaaaaaaaaaaab") == b"aa9aa3b"
    assert R.compress(b"") == b""
    assert R.decompress(b"", 0) == b""
    assert R.decompress(b"", 5, 3) == bytes(8)
    assert R.compress(b"\0") == b"\0" and R.decompress(b"\0", 1) == b"\0"
    for e in dummyfiles["files"]:
        x = committed_file_bytes(e)
        if x is None:
            continue
        y = R.compress(x)
        assert len(y) == e["C"] and sha(y) == e["sha_out"], e["path"]
        # write path (src/filesystemApi.c:767-774): decode with E extra zero bytes, append, re-encode
        z = R.decompress(y, len(x), 1000)
        assert z[:len(x)] == x and z[len(x):] == bytes(1000)
        z = z[:len(x)] + b"tail-bytes" * 100
        assert R.compress(z) == O.encode(z)


def test_dropin_concurrent_threads():
    errors = []

    def worker(t):
        rng = np.random.default_rng(t)
        for k in range(40):
            U = int(rng.integers(0, 200000))
            x = O.gen(int(rng.integers(0, 5)), t * 1000 + k, U)
            y = R.compress(x)
            if y != O.encode(x):
                errors.append(("enc", t, k, U))
            if R.decompress(y, U) != x:
                errors.append(("dec", t, k, U))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[:5]


def test_misaligned_slot_is_rejected():
    d_in = torch.zeros(64, dtype=torch.uint8, device=DEV)
    d_out = torch.zeros(128, dtype=torch.uint8, device=DEV)
    st = torch.full((1,), 0, dtype=torch.int32, device=DEV)
    out_len = torch.zeros(1, dtype=torch.int64, device=DEV)
    R.encode_batch(d_in, _i64([3]), _i64([10]), d_out, _i64([0]), out_len, st)
    torch.cuda.synchronize()
    assert int(st.item()) == R.RLE_STATUS_MISALIGNED


def test_full_size_shard_roundtrip_property():
    """configs[3] per-GPU shape at 1/8 scale (16384 x 64 KiB = 1 GiB): device round trip equal, a
    strided sample (every 1021st buffer) bit-exact vs the oracle, and sum(C) of the sample."""
    n, U = 16384, 65536
    kinds = torch.tensor([i % 4 for i in range(n)], dtype=torch.int32, device=DEV)
    offs = torch.arange(n, dtype=torch.int64, device=DEV) * U
    lens = torch.full((n,), U, dtype=torch.int64, device=DEV)
    d_in = torch.empty(n * U, dtype=torch.uint8, device=DEV)
    R.gen_synthetic(d_in, offs, lens, kinds, None)
    cap = R.round16(R.max_compressed_size(U))
    d_c = torch.empty(n * cap, dtype=torch.uint8, device=DEV)
    coffs = torch.arange(n, dtype=torch.int64, device=DEV) * cap
    clen = torch.zeros(n, dtype=torch.int64, device=DEV)
    R.encode_batch(d_in, offs, lens, d_c, coffs, clen)
    d_out = torch.empty(n * U, dtype=torch.uint8, device=DEV)
    st = torch.full((n,), 0x7777, dtype=torch.int32, device=DEV)
    R.decode_batch(d_c, coffs, clen, d_out, offs, lens, None, st)
    torch.cuda.synchronize()
    assert torch.equal(d_out, d_in)
    assert int((st & 0xFF).abs().sum().item()) == 0
    cl = clen.cpu().numpy()
    for i in range(0, n, 1021):
        x = O.gen(i % 4, i, U)
        y = O.encode(x)
        assert cl[i] == len(y)
        got = d_c[i * cap:i * cap + len(y)].cpu().numpy().tobytes()
        assert got == y, i


def test_configs3_per_rank_shard_full_size():
    """configs[3] at its real per-rank size: 1 M x 64 KiB sharded round-robin over 8 GPUs is 131072 x
    64 KiB = 8 GiB per rank.  Rank 5's shard (global buffer i = 8 k + 5, data kind by local index as
    bench.py's cfg3), generated on device from the global seeds; encode + decode in one launch each.
    Checks: the device round trip is the identity over all 8 GiB, every status is clean, and every
    global buffer i with i % 1021 == 0 in this shard is bit-exact against the
    oracle, stream and size.  Buffers are independent (src/rleCompression.c:9-62 keeps no state
    across calls), so one rank's shard is the whole per-GPU workload."""
    world, rank, n, U = 8, 5, 131072, 65536
    gidx = torch.arange(n, dtype=torch.int64, device=DEV) * world + rank
    kinds = (torch.arange(n, dtype=torch.int32, device=DEV) % 4)
    offs = torch.arange(n, dtype=torch.int64, device=DEV) * U
    lens = torch.full((n,), U, dtype=torch.int64, device=DEV)
    d_in = torch.empty(n * U, dtype=torch.uint8, device=DEV)
    R.gen_synthetic(d_in, offs, lens, kinds, gidx)
    cap = R.round16(R.max_compressed_size(U))
    d_c = torch.empty(n * cap, dtype=torch.uint8, device=DEV)
    coffs = torch.arange(n, dtype=torch.int64, device=DEV) * cap
    clen = torch.zeros(n, dtype=torch.int64, device=DEV)
    est = torch.full((n,), 0x7777, dtype=torch.int32, device=DEV)
    R.encode_batch(d_in, offs, lens, d_c, coffs, clen, est)
    d_out = torch.empty(n * U, dtype=torch.uint8, device=DEV)
    st = torch.full((n,), 0x7777, dtype=torch.int32, device=DEV)
    R.decode_batch(d_c, coffs, clen, d_out, offs, lens, None, st)
    torch.cuda.synchronize()
    assert int(est.abs().sum().item()) == 0
    assert int(st.abs().sum().item()) == 0
    assert torch.equal(d_out, d_in)
    del d_out
    cl = clen.cpu().numpy()
    sample = [k for k in range(n) if (k * world + rank) % 1021 == 0]
    assert len(sample) >= 120
    c_sum = 0
    for k in sample:
        x = O.gen(k % 4, k * world + rank, U)
        assert d_in[k * U:(k + 1) * U].cpu().numpy().tobytes() == x, k
        y = O.encode(x)
        assert cl[k] == len(y), k
        assert d_c[k * cap:k * cap + len(y)].cpu().numpy().tobytes() == y, k
        c_sum += len(y)
    assert c_sum == int(cl[sample].sum())


@pytest.mark.parametrize("seg", [False, True])
def test_decode_status_info_bits(seg):
    # encoder output is status 0, including streams that end in a single 0x00 token (the reference
    # reads it as a pair with the zero padding and fills to U with the zeros it already holds)
    xs = [bytes(4096), b"ab\0", bytes(262144), b"q" * 100 + b"\0", O.gen(1, 3, 70000) + b"\0"]
    ys, _ = gpu_encode(xs, seg=seg)
    dec, st = gpu_decode(ys, [len(x) for x in xs], seg=seg)
    assert dec == xs and (st == 0).all(), st
    # streams that decode short of U: SHORT, the rest zero (src/rleCompression.c:48)
    dec, st = gpu_decode([b"abc", b"ab\0", b"xx9" * 20000], [5, 7, 200000], seg=seg)
    assert list(st) == [R.RLE_STATUS_SHORT] * 3, st
    assert dec[0] == b"abc\0\0" and dec[1] == b"ab" + bytes(5) and dec[2] == b"x" * 180000 + bytes(20000)


def test_large_batch_decode_plain_stores():
    """More than 4096 buffers (plain-store launches): mixed kinds and sizes and streams the encoder
    never emits (serial path), bit-exact against the oracle, twice in a row."""
    rng = np.random.default_rng(21)
    xs = [O.gen(i % 5, i, int(rng.integers(0, 6000))) for i in range(5000)]
    ys = [O.encode(x) for x in xs]
    streams, us, caps = list(ys), [len(x) for x in xs], [len(x) for x in xs]
    for i in range(0, 5000, 997):   # invalid digits / counts past U, with room for the reference's writes
        streams[i] = b"aa:" + ys[i]
        caps[i] = us[i] + 64
    dec, st = gpu_decode(streams, us, caps, poison=False)
    for i in range(5000):
        ref, _ = O.decode(streams[i], us[i], caps[i])
        assert dec[i] == ref, i
    assert all((st[i] & R.RLE_STATUS_SERIAL) for i in range(0, 5000, 997))
    dec2, _ = gpu_decode(streams, us, caps, poison=False)
    assert dec2 == dec


@pytest.mark.parametrize("n", [4097, 4099, 8195, 12288, 16384, 16385])
def test_decode_ragged_batches_past_one_round(n):
    """Batches just past one residency round of the chip (4096 waves): a last round of one to a few
    buffers, XCD-padding workgroups with no buffer, and long / short / serial buffers mixed --
    each buffer decoded exactly once, bit-exact, every status written.  The issue order comes from
    chunk-local sorts of 256 buffers (rle_kernels.hip dec_order_local_kernel), the full chunks
    interleaved and a partial last chunk (n % 256 buffers: 1, 3, 3, 0, 0, 1 here) after them."""
    rng = np.random.default_rng(n)
    sizes = rng.integers(0, 3000, size=n)
    sizes[::7] = 20000   # a few long buffers, so ranges finish unevenly
    xs = [O.gen(i % 5, 7 * i + 1, int(sizes[i])) for i in range(n)]
    streams = [O.encode(x) for x in xs]
    us, caps = [len(x) for x in xs], [len(x) for x in xs]
    for i in range(3, n, 1001):
        streams[i] = b"aa:" + streams[i]
        caps[i] = us[i] + 64
    dec, st = gpu_decode(streams, us, caps)
    for i in range(n):
        ref, _ = O.decode(streams[i], us[i], caps[i])
        assert dec[i] == ref, i
    assert all(st[i] != 0x7777 and (st[i] & R.RLE_STATUS_SERIAL) for i in range(3, n, 1001))
    assert all(st[i] & ~R.RLE_STATUS_SHORT == 0 for i in range(n) if (i - 3) % 1001)


def test_large_decodes_from_threads_and_streams():
    """Large decodes (past one residency round, so each takes an issue-order array) launched by four
    host threads: two on their own streams, two sharing one stream, several times each, with
    growing batch sizes (the per-stream order arrays grow, rle_kernels.hip order_acquire).  Every
    output bit-exact.  The order and decode launches of one call must not interleave with another
    thread's on the shared stream."""
    rng = np.random.default_rng(33)
    n = 9000
    xs = [O.gen(i % 5, 3 * i + 2, int(rng.integers(0, 1500))) for i in range(n)]
    ys = [O.encode(x) for x in xs]
    in_offs, in_total = R.layout([len(y) for y in ys])
    host = np.zeros(in_total, np.uint8)
    for y, o in zip(ys, in_offs):
        host[o:o + len(y)] = np.frombuffer(y, np.uint8)
    d_c = torch.from_numpy(host).to(DEV)
    sizes = [len(x) for x in xs]
    out_offs, out_total = R.layout(sizes)
    want = np.full(out_total, POISON, np.uint8)   # the slots' alignment padding stays poisoned
    for x, o in zip(xs, out_offs):
        want[o:o + len(x)] = np.frombuffer(x, np.uint8)
    coffs, clens, uoffs, ulens = _i64(in_offs), _i64([len(y) for y in ys]), _i64(out_offs), _i64(sizes)
    shared = torch.cuda.Stream(DEV)
    streams = [torch.cuda.Stream(DEV), torch.cuda.Stream(DEV), shared, shared]
    outs = [torch.full((out_total + 16,), POISON, dtype=torch.uint8, device=DEV) for _ in streams]
    stats = [torch.full((n,), 0x7777, dtype=torch.int32, device=DEV) for _ in streams]
    torch.cuda.synchronize()
    errors = []

    def worker(k):
        try:
            for m in (4100, 6000, n, n, 5000):   # prefixes: the order arrays grow, then are reused
                with torch.cuda.stream(streams[k]):
                    R.decode_batch(d_c, coffs[:m], clens[:m], outs[k], uoffs[:m], ulens[:m], None, stats[k][:m],
                                   stream=streams[k])
        except Exception as e:   # noqa: BLE001 (reported below)
            errors.append(repr(e))

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(len(streams))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    torch.cuda.synchronize()
    assert not errors, errors
    for k in range(len(streams)):
        got = outs[k].cpu().numpy()[:out_total]
        assert np.array_equal(got, want), f"thread {k}: decoded bytes differ"
        assert int(stats[k].abs().sum().item()) == 0


def test_large_decodes_per_thread_stream_and_slot_turnover():
    """the issue-order arrays are cached per stream HANDLE.  Two host threads decode large
    batches on hipStreamPerThread (one handle, a different queue in each thread), while a third
    cycles through 20 fresh torch streams (more than the 16 slots: least-recently-used slots are
    handed over, rle_decode_release_stream frees some); every output bit-exact."""
    rng = np.random.default_rng(44)
    n = 6000
    xs = [O.gen(i % 5, 5 * i + 1, int(rng.integers(0, 1800))) for i in range(n)]
    ys = [O.encode(x) for x in xs]
    in_offs, in_total = R.layout([len(y) for y in ys])
    host = np.zeros(in_total, np.uint8)
    for y, o in zip(ys, in_offs):
        host[o:o + len(y)] = np.frombuffer(y, np.uint8)
    d_c = torch.from_numpy(host).to(DEV)
    sizes = [len(x) for x in xs]
    out_offs, out_total = R.layout(sizes)
    want = np.full(out_total, POISON, np.uint8)
    for x, o in zip(xs, out_offs):
        want[o:o + len(x)] = np.frombuffer(x, np.uint8)
    coffs, clens, uoffs, ulens = _i64(in_offs), _i64([len(y) for y in ys]), _i64(out_offs), _i64(sizes)
    nthreads, reps = 3, 6
    outs = [[torch.full((out_total + 16,), POISON, dtype=torch.uint8, device=DEV) for _ in range(reps)]
            for _ in range(nthreads)]
    stats = [[torch.full((n,), 0x7777, dtype=torch.int32, device=DEV) for _ in range(reps)] for _ in range(nthreads)]
    fresh = [torch.cuda.Stream(DEV) for _ in range(20)]
    torch.cuda.synchronize()
    errors = []

    def worker(k):
        try:
            torch.cuda.set_device(0)
            for r in range(reps):
                m = (4200, n, 5000, n, 4500, n)[r]
                if k < 2:
                    R.decode_batch(d_c, coffs[:m], clens[:m], outs[k][r], uoffs[:m], ulens[:m], None, stats[k][r][:m],
                                   stream=R.STREAM_PER_THREAD)
                else:
                    for j, st in enumerate(fresh):
                        R.decode_batch(d_c, coffs[:m], clens[:m], outs[k][r], uoffs[:m], ulens[:m], None,
                                       stats[k][r][:m], stream=st)
                        if j % 3 == 0:
                            R.release_stream(st)
            if k < 2:
                R.release_stream(R.STREAM_PER_THREAD)
        except Exception as e:   # noqa: BLE001 (reported below)
            errors.append(repr(e))

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(nthreads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    torch.cuda.synchronize()
    assert not errors, errors
    for k in range(nthreads):
        for r in range(reps):
            m = (4200, n, 5000, n, 4500, n)[r]
            got = outs[k][r].cpu().numpy()[:out_total]
            end = out_offs[m] if m < n else out_total
            assert np.array_equal(got[:end], want[:end]), f"thread {k} rep {r}: decoded bytes differ"
            assert int(stats[k][r][:m].abs().sum().item()) == 0


@pytest.mark.parametrize("seg", [False, True])
def test_uniform_tiles(seg):
    """Long runs ("v v 9" tokens over whole tiles: the uniform-tile path of rle_device.h
    dec_uniform_tile), every token phase at the tile edges (literal prefixes of 0..6 bytes), bytes
    0x00 / '9' / 0x80 / 0xFF, runs that end anywhere in a tile, next to literals and other runs;
    then streams the encoder never emits: decoded size past U (serial path) and '8' counts."""
    xs = []
    for pre in range(7):
        for v in (0x00, 0x39, 0x80, 0xFF):
            body = bytes([v]) * (9 * 400 * (1 + pre % 3) + pre)
            xs.append(O.gen(1, pre, pre) + body + O.gen(1, 50 + pre, 37) + bytes([v ^ 1]) * (5000 + 13 * pre))
    xs += [bytes(65536), bytes([0x39]) * 100003, O.gen(3, 9, 70000)]
    ys, st = gpu_encode(xs, seg=seg)
    assert (st == 0).all()
    assert ys == [O.encode(x) for x in xs]
    dec, st = gpu_decode(ys, [len(x) for x in xs], seg=seg)
    assert (st == 0).all() and dec == xs
    z = O.encode(bytes(40000))
    streams = [z, z, b"\x00\x008" * 2000, b"\x07\x079" * 1500 + b"ab"]
    us = [30000, 39999, 16000, 13502]
    dec, st = gpu_decode(streams, us, poison=False, seg=seg)
    for i in range(len(streams)):
        ref, _ = O.decode(streams[i], us[i], us[i])
        assert dec[i] == ref, i


@pytest.mark.parametrize("form", ["wave", "seg", "coop"])
def test_phase_map_scan_skip_edges(form):
    """The decode tile skips its phase-map scan when every owned lane's map is constant
    (rle_device.h dec_prepare, RLE_DEC_MAPSKIP).  Streams of "k k k" tokens (a run of k copies of the
    digit k: '2' x 2, '3' x 3, ...) keep the token phase open, so lanes inside such a stretch have
    non-constant maps and the tile takes the scan.  Stretches of 1..400 tokens at every offset
    around lane and tile edges, between random and run-heavy data, decoded in every form (one wave
    per buffer, segmented, cooperative)."""
    def stretch(ntok, first):
        out, k = b"", first
        for _ in range(ntok):
            out += bytes([0x30 + k]) * k
            k = 2 if k == 9 else k + 1
        return out
    xs = []
    for off in list(range(0, 40)) + [1005, 1006, 1007, 1008, 1009, 2015, 2016, 3023, 3024]:
        for ntok in (1, 5, 6, 11, 21, 22, 64, 400):
            xs.append(O.gen(1, off, off) + stretch(ntok, 2 + off % 8) + O.gen(2, ntok, 700) + stretch(ntok // 2 + 1, 5))
    ys = [O.encode(x) for x in xs]
    if form == "coop":
        dec, st = gpu_decode(ys, [len(x) for x in xs], max_in_len=max(len(y) for y in ys),
                             max_out_len=max(len(x) for x in xs))
    else:
        dec, st = gpu_decode(ys, [len(x) for x in xs], seg=(form == "seg"))
    assert (st == 0).all()
    assert dec == xs
    enc, st = gpu_encode(xs, seg=(form == "seg"))
    assert (st == 0).all() and enc == ys
