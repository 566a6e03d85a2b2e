"""The segmented-codec algebra (tests/seg_model.py) against the oracle, on CPU: for many inputs and
segment sizes, the per-segment summaries + per-buffer scan + per-segment writes reassemble exactly
the reference encoding / decoding (src/rleCompression.c:9-62).  This pins the math the multi-wave
kernels (enc_seg_*, dec_seg_*) implement before any GPU runs it."""
import random

import pytest

import seg_model as M
from rle_oracle import decode as o_decode, encode as o_encode


def _segs(n, S):
    return [(p, min(p + S, n)) for p in range(0, n, S)] or [(0, 0)]


def _inputs(rng):
    yield b""
    yield b"a"
    yield bytes(1000)
    yield b"9" * 300                     # '9' runs: '999' tokens, decode phases never converge
    yield b"3" * 31
    yield bytes(rng.getrandbits(8) for _ in range(500))
    for _ in range(60):
        L = rng.randint(1, 700)
        alpha = rng.choice([b"ab", b"a9", b"\0", b"0123456789", bytes(range(256)), b"z"])
        out = bytearray()
        while len(out) < L:
            out += bytes([rng.choice(alpha)]) * rng.choice([1, 1, 2, 3, 8, 9, 10, 17, 40])
        yield bytes(out[:L])


@pytest.mark.parametrize("S", [1, 2, 3, 5, 9, 16, 17, 64, 1008])
def test_encode_segments_reassemble(S):
    rng = random.Random(S)
    for x in _inputs(rng):
        want = o_encode(x)
        plan, total = M.enc_scan(x, _segs(len(x), S))
        assert total == len(want), (S, x[:40])
        got = bytearray(total)
        for (p0, p1), (rs, off, cnt) in zip(_segs(len(x), S), plan):
            piece = M.enc_write(x, p0, p1, rs)
            assert len(piece) == cnt, (S, p0, x[:40])
            got[off:off + cnt] = piece
        assert bytes(got) == want, (S, x[:40])


@pytest.mark.parametrize("S", [1, 2, 3, 4, 7, 16, 64, 1008])
def test_decode_segments_reassemble(S):
    rng = random.Random(100 + S)
    for x in _inputs(rng):
        y = o_encode(x)
        U = len(x)
        plan, total, ok = M.dec_scan(y, _segs(len(y), S))
        assert ok and total == U, (S, x[:40])
        got = bytearray(U)
        for (q0, q1), (e, off) in zip(_segs(len(y), S), plan):
            for pos, v in M.dec_write(y, q0, q1, e, U, off).items():
                got[pos] = v
        assert bytes(got) == o_decode(y, U)[0], (S, x[:40])


def test_decode_final_unbounded_token():
    """a stream whose last token's count digit lies past C (reads the zero padding) fills to U"""
    y = b"ab" + b"cc"
    U = 10
    for S in (1, 2, 3, 4):
        plan, total, ok = M.dec_scan(y, _segs(len(y), S))
        got = bytearray(U)
        for (q0, q1), (e, off) in zip(_segs(len(y), S), plan):
            for pos, v in M.dec_write(y, q0, q1, e, U, off).items():
                got[pos] = v
        assert bytes(got) == o_decode(y, U)[0]
