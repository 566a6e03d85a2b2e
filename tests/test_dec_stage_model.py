"""The decode kernel's staging algebra (tests/dec_stage_model.py) against the oracle, on CPU: for
encoder streams of every data kind the bench uses, staging each 1008-byte tile in one pass (the
product's 192 chunks) or in passes over consecutive lanes (RLE_DEC_CHUNKS 128 / 96 / 16, the
occupancy builds of DESIGN.md §4) decodes to exactly the reference output (src/rleCompression.c:47-62),
and no pass writes outside the staging."""
import random

import pytest

import dec_stage_model as M
from rle_oracle import decode as o_decode, encode as o_encode, gen as o_gen


def _inputs():
    rng = random.Random(20261016)
    yield b"a"
    yield b"aaaaaaaaaaaab"
    yield bytes(5000)                       # zero fill: 3024 B per tile, the staging's worst case
    yield b"9" * 4000                       # '999' tokens
    for kind in range(5):                   # zero / random / runs50 / runs90 / pairs
        for i, size in enumerate((1, 17, 1008, 1009, 4096, 12345)):
            yield o_gen(kind, i, size)
    for _ in range(20):
        L = rng.randint(1, 6000)
        out = bytearray()
        while len(out) < L:
            out += bytes([rng.getrandbits(8)]) * rng.choice([1, 1, 2, 3, 9, 10, 18, 40])
        yield bytes(out[:L])


@pytest.mark.parametrize("chunks", [192, 128, 96, 16])
def test_staged_decode_matches_reference(chunks):
    multi = 0
    for x in _inputs():
        y = o_encode(x)
        got, passes = M.decode_staged(y, len(x), chunks)
        ref, status = o_decode(y, len(x))
        assert status == 0 and got == ref == x
        multi += sum(p > 1 for p in passes)
        if chunks >= 191:
            assert all(p == 1 for p in passes)
    if chunks < 191:
        assert multi > 0, "the inputs must exercise the pass split"
