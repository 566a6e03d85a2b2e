"""GPU parity of the large-batch decode in rounds (csrc/rle_round.h dec_round_kernel: one
workgroup per buffer, its waves on consecutive tiles, the token phase and the output offset of
src/rleCompression.c:50-60 crossing tiles through LDS) against the oracle, at every round width
(4, 8 and 16 waves).  Batches have more than 4096 buffers and a largest stream of at least 8 decode
tiles, so the sized entry point takes the round kernel: synthetic kinds at ragged sizes, crafted
literal / "vv2" / run-heavy streams with pairs across tile edges, single-value tiles, the reference's
invalid streams (the exact serial path), empty and one-byte streams, exact / short / overflow U.
Bit-exact; output slots poisoned (a byte written past U shows up)."""
import numpy as np
import pytest

import rle_mi355x as R
import rle_oracle as O
from test_gpu_fastpath import _cases, _natural_size, _pairs_data
from test_gpu_parity import gpu_decode

pytestmark = pytest.mark.gpu
NMIN = 4097            # past one residency round (csrc/rle_kernels.hip kDecRound)
ROUND_MIN_IN = 8064    # 8 decode tiles: the round kernel's threshold (kRoundMinIn)


@pytest.fixture(params=[4, 8, 16])
def round_waves(request):
    prev = R.set_dec_round(request.param)
    yield request.param
    R.set_dec_round(prev)


def _filler(rng, k):
    """k encoder streams of 8-20 KiB random / runs50 data (keeps the batch past 4096 buffers and its
    largest stream past the round threshold)."""
    xs = [O.gen(1 + (i % 2), 50000 + i, int(rng.integers(ROUND_MIN_IN, 20000))) for i in range(k)]
    return xs, [O.encode(x) for x in xs]


def _decode_check(streams, us, caps=None, seed=0):
    """Decode streams (+ filler) in one launch through the round kernel and compare every buffer with
    the oracle's decode (U bytes, then the cap's tail poisoned as the oracle leaves it untouched)."""
    rng = np.random.default_rng(seed)
    caps = list(caps) if caps is not None else list(us)
    k = max(0, NMIN - len(streams))
    fx, fy = _filler(rng, max(k, 1))
    allys = list(streams) + fy
    allus = list(us) + [len(x) for x in fx]
    allcaps = caps + [len(x) for x in fx]
    mi = max(len(y) for y in allys)
    assert mi >= ROUND_MIN_IN and len(allys) >= NMIN
    dec, st = gpu_decode(allys, allus, allcaps, max_in_len=mi, max_out_len=max(allus))
    for i, y in enumerate(streams):
        ref, rst = O.decode(y, us[i], caps[i])
        assert dec[i] == ref, (i, len(y), us[i], caps[i])
    for j, x in enumerate(fx):
        assert dec[len(streams) + j] == x, j
    return st


def test_round_synthetic_kinds(round_waves):
    """Every synthetic kind (zero, random, runs50, runs90, pairs) at ragged sizes up to 66 KiB."""
    rng = np.random.default_rng(round_waves)
    xs = []
    for i in range(NMIN + 40):
        n = int(rng.integers(1, 66000)) if i % 7 else 65536
        xs.append(O.gen(i % 5, 9000 + i, n))
    ys = [O.encode(x) for x in xs]
    st = _decode_check(ys, [len(x) for x in xs], seed=1)
    assert ((st[:len(xs)] & 0xFF) == 0).all()


def test_round_crafted_literal_pair_and_run_tiles(round_waves):
    """Literal / "vv2" streams with pairs at the last owned positions of tiles, other counts and
    run-heavy stretches (the literal, general and two-pass general tile paths side by side in one
    round), decoded at their natural size, 5 bytes more (SHORT: zero fill) and 3 fewer (the serial
    path: OVERFLOW)."""
    cases = _cases()
    ys = [s for s, _ in cases]
    nat = [_natural_size(s) for s in ys]
    for delta in (0, 5, -3):
        us = [max(0, u + delta) for u in nat]
        _decode_check(ys * 4, us * 4, seed=20 + delta)


def test_round_single_value_and_uniform_tiles(round_waves):
    """Long runs of one byte ("v v 9" tokens: the uniform test and the single-value fill) entered at
    every phase and ending around tile edges, next to literal tiles, and runs of different bytes."""
    rng = np.random.default_rng(9)
    xs = []
    for n in [1008 * k + d for k in range(1, 9) for d in (-40, -9, -1, 0, 1, 9, 333)]:
        for lead in (0, 1, 5, 17, 1008, 3000):
            x = bytearray(_pairs_data(rng, n + lead + 500, 0.02))
            v = int(rng.integers(0, 256))
            x[lead:lead + n * 3] = bytes([v]) * min(n * 3, len(x) - lead)
            xs.append(bytes(x[: lead + n * 3 + 200]))
    for i in range(60):
        n = int(rng.integers(1, 200000))
        lens = rng.integers(1, 30000, size=16)
        xs.append(np.repeat(rng.integers(0, 256, size=16).astype(np.uint8), lens)[:n].tobytes())
    ys = [O.encode(x) for x in xs]
    for delta in (0, 7):
        us = [len(x) + delta for x in xs]
        _decode_check(ys * 6, us * 6, seed=3 + delta)


def test_round_invalid_streams_match_reference(vectors, round_waves):
    """The compiled reference's decodes of invalid streams (counts outside '1'..'9', unbounded
    counts, streams longer than U + E): the exact serial path inside the round kernel."""
    cases = vectors["invalid_decode"]
    streams = [bytes.fromhex(v["in"]) for v in cases]
    us = [v["U"] for v in cases]
    caps = [v["U"] + v["E"] for v in cases]
    rng = np.random.default_rng(4)
    fx, fy = _filler(rng, NMIN)
    allys = streams + fy
    dec, st = gpu_decode(allys, us + [len(x) for x in fx], caps + [len(x) for x in fx], poison=False,
                         max_in_len=max(len(y) for y in allys), max_out_len=max(us + [len(x) for x in fx]))
    bad = [i for i in range(len(cases)) if dec[i] != bytes.fromhex(cases[i]["out"])]
    assert not bad, (len(bad), cases[bad[0]], dec[bad[0]].hex())
    assert ((st & 0xFF) == 0).all()
    for j, x in enumerate(fx):
        assert dec[len(streams) + j] == x, j


def test_round_edge_streams(round_waves):
    """Empty streams (U = 0 and U > 0), one-byte streams ("\\0" ends in an unbounded token), streams
    of exactly 1, 8 and 16 tiles (rounds that end full), and one tile past a round."""
    rng = np.random.default_rng(5)
    ys, us = [], []
    for U in (0, 1, 5, 100):
        ys.append(b"")
        us.append(U)
    for b in (b"\x00", b"\x01", b"a", b"aa2", b"aa9aa3b"):
        for U in (len(b), len(b) + 3):
            ys.append(b)
            us.append(U)
    for tiles in (1, 2, 4, 7, 8, 9, 15, 16, 17, 24, 33):
        for d in (-2, 0, 1):
            n = 1008 * tiles + d
            y = O.encode(_pairs_data(rng, n, 0.0))   # literals only: C == U
            ys.append(y)
            us.append(len(y))
    st = _decode_check(ys * 40, us * 40, seed=6)
    assert (st[:len(ys) * 40] >= 0).all()
