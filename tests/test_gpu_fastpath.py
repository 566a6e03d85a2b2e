"""GPU parity of the decode's literal-tile fast path (csrc/rle_device.h dec_tile_fast) against
the oracle: crafted streams of literals and "vv2" pairs, the tiles the fast path takes, mixed with
pairs of other counts and run-heavy stretches (tiles the general path takes), with pairs placed
across tile edges, ragged tails, and decoded sizes that are exact, too large (SHORT: zero fill) or
too small (OVERFLOW: the serial path).  Bit-exact, slots poisoned."""
import numpy as np
import pytest

import rle_oracle as O
from test_gpu_parity import gpu_decode

pytestmark = pytest.mark.gpu
STEP = 1008   # decode tile step (csrc/rle_device.h kTileStep)


def _stream(rng, n_bytes, p_pair, p_other, p_run, forced=()):
    """Token stream of about n_bytes: literals, pairs "vv2", pairs with another count digit
    (p_other), and short run-heavy stretches (p_run).  Each token's byte differs from the byte
    before it, so the decoder's parse is exactly these tokens.  forced: positions where a "vv2"
    pair must start (when the stream reaches them at a token boundary, else the next one).
    Returns (stream, decoded length)."""
    out = bytearray()
    U = 0
    forced = sorted(forced)
    fi = 0
    prev = -1
    while len(out) < n_bytes:
        v = int(rng.integers(0, 256))
        while v == prev:
            v = int(rng.integers(0, 256))
        want_pair = fi < len(forced) and len(out) >= forced[fi]
        if want_pair:
            fi += 1
        r = rng.random()
        if want_pair or r < p_pair:
            out += bytes([v, v, ord("2")])
            U += 2
            prev = ord("2")
        elif r < p_pair + p_other:
            c = int(rng.integers(3, 10))
            out += bytes([v, v, ord("0") + c])
            U += c
            prev = ord("0") + c
        elif r < p_pair + p_other + p_run:
            for _ in range(int(rng.integers(2, 12))):
                c = int(rng.integers(2, 10))
                out += bytes([v, v, ord("0") + c])
                U += c
                prev = ord("0") + c
                v = (v + 1 + int(rng.integers(0, 254))) % 256
                while v == prev:
                    v = (v + 1) % 256
        else:
            out += bytes([v])
            U += 1
            prev = v
    return bytes(out), U


def _cases():
    rng = np.random.default_rng(2024)
    cases = []
    lengths = [STEP * k + d for k in range(1, 7) for d in (-20, -3, -2, -1, 0, 1, 2, 3, 17)]
    lengths += [int(x) for x in rng.integers(1, 7000, size=120)]
    for i, n in enumerate(lengths):
        p_pair = (0.0, 0.02, 0.1, 0.2, 0.35)[i % 5]
        p_other = (0.0, 0.0, 0.0005, 0.01)[i % 4]
        p_run = (0.0, 0.0, 0.0, 0.002)[(i // 4) % 4]
        cases.append(_stream(rng, n, p_pair, p_other, p_run))
    # pairs starting at the last owned positions of a tile and just before them
    for k in (1, 2, 3):
        for back in (1, 2, 3, 4):
            cases.append(_stream(rng, STEP * k + 500, 0.02, 0.0, 0.0, forced=(STEP * k - back,)))
            cases.append(_stream(rng, STEP * (k + 1) + 40, 0.0, 0.0, 0.0, forced=(STEP * k - back, STEP * k + 1)))
    # a general first tile (count 5) handing a partial chunk to literal tiles, and back
    for j in range(20):
        cases.append(_stream(rng, 4000 + 37 * j, 0.05, 0.0, 0.0, forced=()))
        s, U = cases[-1]
        cases[-1] = (bytes([65, 65, ord("5")]) + s[1:] if s[0] != 65 else s, None)
    return cases


def _natural_size(s):
    """Decoded length of a stream whose tokens are all bounded (the generator's streams)."""
    U, j = 0, 0
    while j < len(s):
        if j + 1 < len(s) and s[j] == s[j + 1]:
            U += s[j + 2] - ord("0") if j + 2 < len(s) else 0
            j += 3
        else:
            U += 1
            j += 1
    return U


def test_literal_tiles_match_oracle():
    cases = _cases()
    streams = [s for s, _ in cases]
    sizes = [_natural_size(s) for s in streams]
    for delta in (0, 7, -5):   # exact, SHORT (zero fill), OVERFLOW (serial path)
        us = [max(0, u + delta) for u in sizes]
        dec, st = gpu_decode(streams, us)
        for i, s in enumerate(streams):
            ref, rst = O.decode(s, us[i])
            assert dec[i] == ref, (delta, i, len(s), us[i])
        if delta == 0:
            assert ((st & 0xFF) == 0).all()


def test_literal_tiles_encoder_output_batch():
    """Encoder output of text-like data (doubled letters are "vv2" pairs): the bench's random kind
    and literal-heavy tiles with a few pairs per lane, decoded in one batch."""
    rng = np.random.default_rng(7)
    xs = []
    for i in range(400):
        n = int(rng.integers(1, 20000))
        alpha = np.frombuffer(b"etaoinshrdlucmfwypvbgkqjxz ", np.uint8)
        x = rng.choice(alpha, size=n)
        dup = rng.random(n) < (0.02, 0.05, 0.1)[i % 3]
        x = np.repeat(x, np.where(dup, 2, 1))[:n]
        xs.append(x.tobytes())
    ys = [O.encode(x) for x in xs]
    dec, st = gpu_decode(ys, [len(x) for x in xs])
    bad = [i for i in range(len(xs)) if dec[i] != xs[i]]
    assert not bad, (len(bad), bad[:5])
    assert ((st & 0xFF) == 0).all()


def _pairs_data(rng, n, p_dup, p_triple=0.0, forced=()):
    """Bytes with no equal neighbours except doubled bytes (p_dup per byte), the odd triple
    (p_triple: a tile the encoder's fast path declines), and doubles at the forced positions."""
    x = rng.integers(0, 255, size=n, dtype=np.int64)
    x = np.where(x >= np.roll(x, 1), x + 1, x)      # break most accidental repeats
    x[1:] = np.where(x[1:] == x[:-1], (x[1:] + 1) % 256, x[1:])
    x = x.astype(np.uint8)
    dup = rng.random(n) < p_dup
    tri = rng.random(n) < p_triple
    y = np.repeat(x, np.where(tri, 3, np.where(dup, 2, 1)))[:n].copy()
    for f in forced:   # a pair starting exactly at f, then a different byte
        if 0 < f and f + 2 < n:
            y[f] = y[f - 1] ^ 0x55
            y[f + 1] = y[f]
            y[f + 2] = y[f] ^ 0x0F
    return y.tobytes()


def test_literal_tiles_encode_match_oracle():
    """Encoder fast path (csrc/rle_device.h enc_tile_fast): literal and pair tiles, pairs at the
    edges of 1024-byte tiles (buffers <= 16 KiB) and 1008-byte tiles (larger), runs of 3 that
    make a tile decline, ragged sizes; output bit-exact and nothing written past C."""
    from test_gpu_parity import _oracle_parity
    rng = np.random.default_rng(11)
    xs = []
    for i in range(300):
        n = int(rng.integers(1, 40000))
        xs.append(_pairs_data(rng, n, (0.0, 0.01, 0.05, 0.12, 0.3)[i % 5], (0.0, 0.0, 0.0002, 0.003)[i % 4]))
    for k in range(1, 8):
        for d in (-3, -2, -1, 0, 1):
            xs.append(_pairs_data(rng, 1024 * k + 300, 0.01, forced=(1024 * k + d,)))
            xs.append(_pairs_data(rng, 17000 + 1008 * k, 0.01, forced=(1008 * k + d, 1008 * k + d + 5)))
            xs.append(_pairs_data(rng, 1024 * k + d + 2, 0.02))
    _oracle_parity(xs)


def test_run_tiles_encode_match_oracle():
    """Encoder run tiles (csrc/rle_device.h enc_tile_run): runs spanning whole tiles, starting at
    every phase mod 9 before a tile edge and ending 0..10 bytes past one (the last token's count
    from the lookahead bits, a lone byte for count 1), runs of 0x00 and of digits, literal and pair
    tiles after them (the staged partial chunk handed over), both tile forms (<= 16 KiB: 1024-byte
    tiles, larger: 1008)."""
    from test_gpu_parity import _oracle_parity
    rng = np.random.default_rng(5)
    xs = []
    for step, base in ((1024, 0), (1008, 17000)):
        for k in (1, 2, 3):
            edge = base + step * k
            for start_back in (0, 1, 4, 8, 9, 17, 700):
                for end_past in (0, 1, 2, 7, 8, 9, 10):
                    n = edge + 2500
                    x = bytearray(_pairs_data(rng, n, 0.03))
                    s0 = max(0, edge - step - start_back)
                    e0 = min(n, edge + end_past)
                    v = (0x00, ord("9"), 0x41)[(k + end_past) % 3]
                    x[s0:e0] = bytes([v]) * (e0 - s0)
                    if e0 < n and x[e0] == v:
                        x[e0] = v ^ 1
                    xs.append(bytes(x))
    for i in range(60):   # long runs of random lengths, random values, ragged sizes
        n = int(rng.integers(1, 60000))
        lens = rng.integers(1, 5000, size=64)
        vals = rng.integers(0, 4, size=64)
        xs.append(np.repeat(vals.astype(np.uint8), lens)[:n].tobytes())
    _oracle_parity(xs)


def test_single_value_tiles_decode_match_oracle():
    """Decoder single-value tiles (csrc/rle_device.h dec_tile_fill): long runs of one byte (count-9
    pair tokens, >= 2.86x expansion) entered with every staged partial length, ending at every
    offset around tile edges, followed by literal tiles, ragged sizes, exact / short / overflow U."""
    rng = np.random.default_rng(9)
    xs = []
    for n in [1008 * k + d for k in range(1, 6) for d in (-40, -9, -1, 0, 1, 9, 333)]:
        for lead in (0, 1, 5, 15, 16, 17, 31):
            x = bytearray(_pairs_data(rng, n + lead + 500, 0.02))
            v = int(rng.integers(0, 256))
            x[lead:lead + n * 3] = bytes([v]) * min(n * 3, len(x) - lead)
            xs.append(bytes(x[: lead + n * 3 + 200]))
    for i in range(40):
        n = int(rng.integers(1, 200000))
        lens = rng.integers(1, 30000, size=16)
        xs.append(np.repeat(rng.integers(0, 256, size=16).astype(np.uint8), lens)[:n].tobytes())
    ys = [O.encode(x) for x in xs]
    for delta in (0, 5, -3):
        us = [max(0, len(x) + delta) for x in xs]
        dec, st = gpu_decode(ys, us)
        for i, y in enumerate(ys):
            ref, _ = O.decode(y, us[i])
            assert dec[i] == ref, (delta, i, len(xs[i]))


def test_consecutive_single_value_tiles_decode_match_oracle():
    """Whole uniform tiles back to back (RLE_DEC_VRUN, csrc/rle_device.h dec_fill_run): runs of
    3024 k bytes ("v v 9" tokens filling whole 1008-byte tiles) of the same or of different bytes,
    aligned on tile edges by literal leads of whole tiles, then off the edges, with general and
    literal tiles between them; 1 and 4500 buffers (both decode kernels), exact / short / overflow U."""
    rng = np.random.default_rng(31)

    def literals(n):
        x = rng.integers(0, 255, size=n).astype(np.uint8)
        for i in range(1, n):   # no two equal neighbours: n literal tokens
            if x[i] == x[i - 1]:
                x[i] = (x[i] + 1) % 255
        return x.tobytes()

    xs = []
    for lead in (0, 1008, 2016, 1, 17, 1000):
        for ks in ((1, 1), (2, 3), (1, 1, 1, 1), (3, 1, 2)):
            for same in (True, False):
                x = bytearray(literals(lead))
                v = int(rng.integers(0, 256))
                for k in ks:
                    if not same:
                        v = (v + 1 + int(rng.integers(0, 254))) % 256
                    x += bytes([v]) * (3024 * k)
                x += literals(int(rng.integers(0, 3000)))
                xs.append(bytes(x))
    for i in range(40):   # uniform tiles, then run-heavy / literal stretches, then uniform again
        parts = []
        for _ in range(6):
            r = rng.random()
            if r < 0.5:
                parts.append(bytes([int(rng.integers(0, 256))]) * (3024 * int(rng.integers(1, 4)) + int(rng.integers(0, 3))))
            elif r < 0.75:
                parts.append(literals(int(rng.integers(1, 2500))))
            else:
                parts.append(O.gen(2, 900 + i, int(rng.integers(1, 4000))))
        xs.append(b"".join(parts))
    ys = [O.encode(x) for x in xs]
    for delta in (0, 7, -5):
        us = [max(0, len(x) + delta) for x in xs]
        dec, st = gpu_decode(ys, us)
        for i, y in enumerate(ys):
            ref, _ = O.decode(y, us[i])
            assert dec[i] == ref, (delta, i, len(xs[i]))
    # the large-batch kernel (96-chunk staging, > 4096 buffers)
    big = (xs * (4500 // len(xs) + 1))[:4500]
    ybig = [O.encode(x) for x in big]
    dec, st = gpu_decode(ybig, [len(x) for x in big])
    for i, x in enumerate(big):
        assert dec[i] == x, i


def test_large_batch_small_staging_matches_oracle():
    """Batches past one residency round (> 4096 buffers) decode with the 96-chunk staging
    (csrc/rle_kernels.hip decode_kernel<kDecChunksLarge>), where output-heavy general tiles (runs of
    mixed values) stage in two passes: every data kind, ragged sizes, bit-exact."""
    from test_gpu_parity import _oracle_parity
    rng = np.random.default_rng(21)
    xs = []
    for i in range(4400):
        kind = i % 6
        n = int(rng.integers(1, 9000))
        if kind < 4:
            xs.append(O.gen(kind, 7000 + i, n))
        elif kind == 4:   # runs of 8-9 of changing values: ~2.9x expansion, not single-valued
            lens = rng.integers(8, 10, size=n // 8 + 2)
            xs.append(np.repeat(rng.integers(0, 256, size=len(lens)).astype(np.uint8), lens)[:n].tobytes())
        else:
            xs.append(_pairs_data(rng, n, 0.05))
    _oracle_parity(xs)


def test_literal_last_tiles_encode_match_oracle():
    """Encoder literal path on the buffer's last tile (enc_tile_fast<k64, true>: stores clipped at
    C, the last 4 bytes stored again): every size around the tile forms' edges, pairs in the last
    bytes, a pair ending exactly at U, and nothing written past C (the slots are poisoned)."""
    from test_gpu_parity import _oracle_parity
    rng = np.random.default_rng(33)
    xs = []
    for n in list(range(1, 80)) + [1024 * k + d for k in range(1, 5) for d in range(-6, 7)] + \
            [17000 + 1008 * k + d for k in range(0, 3) for d in (-3, -1, 0, 1, 5)]:
        for p_dup in (0.0, 0.03, 0.2):
            x = bytearray(_pairs_data(rng, n, p_dup))
            xs.append(bytes(x))
            if n >= 3:   # a pair as the last two bytes, and one just before them
                y = bytearray(x)
                y[-1] = y[-2]
                if n >= 4 and y[-3] == y[-2]:
                    y[-3] ^= 0x5A
                xs.append(bytes(y))
    _oracle_parity(xs)


def test_periodic_tiles_decode_match_oracle():
    """Periodic streams ("v v 9" tokens of one byte v: v = 0x00, '9', '0', random), which the
    single-value tiles decode (dec_tile_fill), entered at every phase (a 1- or 3-byte token first),
    and the same streams with the pattern broken once -- another count digit, another byte at a
    token start, a literal, a stray byte -- at positions all over a tile and at its edges, so that
    the general path decodes those tiles; also U short of / past the decoded length.  (Round 3 also
    tried a dedicated periodic-tile path ahead of the phase scan: slower)"""
    rng = np.random.default_rng(33)
    ys = []
    for v in (0x00, 0x39, 0x30, 0x61, int(rng.integers(0, 256))):
        tok = bytes([v, v, 0x39])
        for lead in (b"", b"\x01", b"\x02\x02\x35", b"\x07", b"\x03\x03\x32\x04"):
            base = lead + tok * 1400   # ~4 tiles of tokens
            ys.append(base)
            for p in (len(lead), len(lead) + 1, len(lead) + 2, 500, 1006, 1007, 1008, 1009, 1010, 1500,
                      2015, 2016, 2017, 3023, 3024, 3025, len(base) - 5):
                for b in (0x38, v ^ 0x40, 0x31, 0x00):
                    y = bytearray(base)
                    y[p] = b
                    ys.append(bytes(y))
                y = bytearray(base)   # a literal inserted
                ys.append(bytes(y[:p]) + bytes([v ^ 0x55]) + bytes(y[p:]))
    def size(s):   # the decoded length with counts clamped to 1..9 (the oracle decides the rest)
        U, j = 0, 0
        while j < len(s):
            if j + 1 < len(s) and s[j] == s[j + 1]:
                U += min(9, max(1, s[j + 2] - 48)) if j + 2 < len(s) else 1
                j += 3
            else:
                U += 1
                j += 1
        return U

    us = [size(y) for y in ys]
    for delta in (0, -7, 4):
        uu = [max(0, u + delta) for u in us]
        dec, st = gpu_decode(ys, uu)
        for i, y in enumerate(ys):
            ref, _ = O.decode(y, uu[i])
            assert dec[i] == ref, (delta, i)


def test_encode_tile_pairs_match_oracle():
    """Two encode tiles per step (csrc/rle_device.h enc_pair, buffers up to 16 KiB): every tile count
    1..16 with the last tile 1..4 bytes, a few hundred, or full; pairs of run tiles (one run over
    both, a boundary at the first byte, the run ending at, before and 1..9 bytes past the pair's
    end), literal pairs (pairs of equal bytes straddling the two tiles and the pair's end, the
    second tile the buffer's last with < 4, 4..16 and more output bytes), and every mix of run,
    literal and general tiles within a pair; against the oracle."""
    from test_gpu_parity import _oracle_parity
    rng = np.random.default_rng(77)
    xs = []
    for nt in range(1, 17):
        for last in (1, 2, 3, 4, 5, 300, 1023, 1024):
            n = 1024 * (nt - 1) + last
            for kind in (0, 1, 2, 3):
                xs.append(O.gen(kind, 1000 * nt + last + kind, n))
            xs.append(_pairs_data(rng, n, 0.06))
    for k in (1, 2, 3, 6):   # pair boundaries at 2048 k
        edge = 2048 * k
        for back in range(0, 4):
            for fwd in range(0, 11):
                x = bytearray(_pairs_data(rng, edge + 600, 0.05))
                # a run over the pair before the edge, ending fwd bytes past it
                s0 = max(0, edge - 2048 - back)
                x[s0:edge + fwd] = bytes([0x5A]) * (edge + fwd - s0)
                if edge + fwd < len(x) and x[edge + fwd] == 0x5A:
                    x[edge + fwd] = 0x5B
                xs.append(bytes(x))
                # a pair of equal bytes straddling the tiles' edges
                y = bytearray(_pairs_data(rng, edge + 1024 + 3, 0.0))
                for e in (edge - 1024, edge):
                    if 1 <= e - back < len(y):
                        y[e - back] = y[e - back - 1]
                xs.append(bytes(y))
    for i in range(200):   # run / literal / general tiles mixed inside pairs
        n = int(rng.integers(1, 16385))
        x = bytearray(_pairs_data(rng, n, float(rng.choice([0.0, 0.02, 0.2]))))
        for _ in range(int(rng.integers(0, 4))):
            a = int(rng.integers(0, n))
            b = min(n, a + int(rng.integers(1, 3000)))
            x[a:b] = bytes([int(rng.integers(0, 256))]) * (b - a)
        xs.append(bytes(x))
    _oracle_parity(xs)


def test_decode_tile_pairs_match_oracle():
    """Two decode tiles per step in the one-round kernel (csrc/rle_device.h dec_pair): streams built
    tile by tile from literal stretches ("vv2" pairs, the fast path's tiles) and general stretches
    (a count other than 2, or run tokens), in every pattern of 1..9 tiles, so that every pair is
    literal + literal, literal + general, general + literal (a staged partial chunk handed to a
    literal pair) or general + general, the last tile of an odd count alone, and the last tile a
    tail; shifted by 0..4 bytes so that tokens straddle the pair's and the tiles' edges.  Decoded in
    one batch (one-round kernel) at the exact size, a larger one (SHORT) and a smaller one (the serial
    path), against the oracle."""
    rng = np.random.default_rng(4242)
    streams = []
    for nt in range(1, 10):
        for pat in range(min(1 << nt, 48)):
            bits = pat if nt <= 5 else int(rng.integers(0, 1 << nt))
            for shift in (0, 1, 2, 3, 4) if nt <= 4 else (int(rng.integers(0, 5)),):
                parts = [bytes(range(1, 1 + shift))]
                for t in range(nt):
                    general = (bits >> t) & 1
                    n = STEP - (int(rng.integers(0, 40)) if t == nt - 1 else 0)
                    s, _ = _stream(rng, n, 0.06, 0.01 if general else 0.0, 0.002 if general else 0.0)
                    if general:   # at least one "vv5" token in the tile
                        s = s[:200] + bytes([0x37, 0x37, ord("5")]) + s[203:] if s[199] != 0x37 else s
                    parts.append(s[:n])
                streams.append(b"".join(parts))
    # a token boundary is not preserved across the parts' joins: decode whatever the bytes parse to
    sizes = [_natural_size(s) for s in streams]
    assert len(streams) <= 4096
    for delta in (0, 9, -4):
        us = [max(0, u + delta) for u in sizes]
        dec, st = gpu_decode(streams, us)
        for i, s in enumerate(streams):
            ref, rst = O.decode(s, us[i])
            assert dec[i] == ref, (delta, i, len(s), us[i])
