"""GPU parity of the cooperative small-buffer kernels (csrc/rle_coop.hip: one workgroup per buffer,
one wave per tile), reached through the sized entry points of include/rle_mi355x.h, against the
oracle and the compiled reference's golden vectors.  Bit-exact everywhere, slots poisoned.

The size hints choose the kernel; a hint smaller than a buffer (allowed only here, to reach the
path) sends that buffer to the workgroup's one-wave fallback, so both paths of the kernel run."""
import numpy as np
import pytest

import rle_oracle as O
from test_gpu_parity import gpu_decode, gpu_encode

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, scope="module")
def _always_coop():
    # the launcher's default takes the cooperative kernels only for launches resident at once;
    # these tests run them for every batch (the library's test setter, not the environment)
    import rle_mi355x as R
    R.set_coop_mode(1)
    yield
    R.set_coop_mode(-1)


def _hints(xs, ys):
    return max(len(x) for x in xs), max(len(y) for y in ys), max(len(x) for x in xs)


def coop_parity(xs, enc_hint=None, dec_hints=None):
    """Encode with the sized entry point, compare with the oracle, decode the oracle's streams with
    the sized entry point, compare with the input."""
    refs = [O.encode(x) for x in xs]
    mx = max(1, max(len(x) for x in xs))
    ys, st = gpu_encode(xs, max_len=enc_hint if enc_hint is not None else mx)
    assert (st == 0).all()
    bad = [i for i in range(len(xs)) if ys[i] != refs[i]]
    assert not bad, (len(bad), bad[:3], [len(xs[i]) for i in bad[:3]])
    mi = max(1, max(len(y) for y in refs))
    hi, ho = dec_hints if dec_hints is not None else (mi, mx)
    dec, st = gpu_decode(refs, [len(x) for x in xs], max_in_len=hi, max_out_len=ho)
    bad = [i for i in range(len(xs)) if dec[i] != xs[i]]
    assert not bad, (len(bad), bad[:3], [len(xs[i]) for i in bad[:3]])
    assert ((st & 0xFF) == 0).all()


def test_config1_shape():
    # BASELINE configs[1]: 4096 x 4 KiB random / zero
    coop_parity([O.gen(1 if i % 2 == 0 else 0, i, 4096) for i in range(4096)])


@pytest.mark.parametrize("kind", [0, 1, 2, 3, 4])
def test_every_kind_and_small_size(kind):
    sizes = [0, 1, 2, 15, 16, 17, 1007, 1008, 1009, 1023, 1024, 1025, 2016, 2017, 2048, 2049, 3024, 3072, 4095,
             4096, 4097, 5000, 6143, 6144, 7000, 8191, 8192]
    coop_parity([O.gen(kind, 7 * kind + i, s) for i, s in enumerate(sizes)])


@pytest.mark.parametrize("kind", [0, 1, 2, 3, 4])
def test_every_kind_nine_to_sixteen_tiles(kind):
    # 12- and 16-wave workgroups (encode up to 16 KiB; decode up to 16128 stream bytes); streams
    # longer than that (random 16 KiB) take the workgroup's one-wave fallback under the hint
    sizes = [8193, 9216, 10000, 11000, 12287, 12288, 12289, 13000, 15000, 16127, 16128, 16129, 16383, 16384]
    xs = [O.gen(kind, 11 * kind + i, s) for i, s in enumerate(sizes)]
    coop_parity(xs, dec_hints=(16128, 16384))


@pytest.mark.parametrize("kind", [0, 3])
def test_compressible_sixteen_to_thirtytwo_kib_decode(kind):
    # decode staging of 32 KiB (4-, 8- and 16-wave workgroups, one round): compressible buffers of
    # 16-32 KiB, zero runs crossing the staging's 16 KiB half, and exact-length / ragged ends; then
    # with a literal-heavy buffer in the batch (22 tiles: three rounds)
    sizes = [16385, 17000, 20000, 24576, 30000, 32767, 32768]
    xs = [O.gen(kind, 5 * kind + i, s) for i, s in enumerate(sizes)]
    xs += [b"\0" * 32768, b"\0" * 16000 + b"x" * 300 + b"\0" * 16468]
    mi = max(len(O.encode(x)) for x in xs)
    assert mi <= 16128, mi
    coop_parity(xs, enc_hint=16384, dec_hints=(mi, 32768))
    xs.append(b"ab" * 8000 + b"\0" * 16768)
    coop_parity(xs, dec_hints=(max(len(O.encode(x)) for x in xs), 32768))


@pytest.mark.parametrize("kind", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("umax", [16384, 32768, 65536])
def test_rounds_of_sixteen_tiles(kind, umax):
    """Rounds of 16 waves (rle_coop_limits.h): encode 17-64 tiles (2 and 4 rounds), decode 17-80
    tiles into 16 / 32 / 64 KiB staging; sizes at the round edges (16 x 1024 encode, 16 x 1008
    decode), with the batch's own hints and with the largest hints of the staging (buffers past the
    rounds: the workgroup's one-wave fallback)."""
    sizes = [1500, 8000, 16000, 16128, 16129, 16384, 16385, 20000, 24576, 32256, 32257, 32767, 32768, 40000,
             48384, 48385, 50000, 64512, 65535, 65536]
    xs = [O.gen(kind, 13 * kind + i, s) for i, s in enumerate(s for s in sizes if s <= umax)]
    coop_parity(xs)
    coop_parity(xs, dec_hints=(1008 * 16 * (2 if umax == 16384 else 3 if umax == 32768 else 5), umax))


def test_rounds_invalid_streams_take_serial_decoder():
    # a stream the tiled path declines only in a later round (a bad digit past 16 tiles), a stream
    # that decodes past U in a later round, and a valid one in the same batch
    x = O.gen(3, 5, 60000)
    y = bytearray(O.encode(x))
    z = bytearray(y)
    k = len(z) - 40
    while not (0x31 <= z[k] <= 0x39 and z[k - 1] == z[k - 2]):
        k -= 1
    z[k] = ord(":")   # a count byte past '9': not encoder output
    streams = [bytes(y), bytes(z), bytes(y) + b"ab" * 100]
    us = [len(x), len(x), len(x)]
    caps = [len(x), len(x) + 32, len(x) + 32]
    dec, st = gpu_decode(streams, us, caps, poison=False, max_in_len=max(len(s) for s in streams),
                         max_out_len=max(us))
    for i, (s, u, c) in enumerate(zip(streams, us, caps)):
        ref, rst = O.decode(s, u, c)
        assert dec[i] == ref, i
    import rle_mi355x as R
    assert st[0] == 0 and st[2] & R.RLE_STATUS_SERIAL and st[2] & R.RLE_STATUS_OVERFLOW, st


def test_runs_and_digits_across_tile_edges():
    # runs that end or cross a tile edge (1008 k decode, 1024 k encode) by 1..10 bytes, digit bytes
    xs = []
    for k in range(1, 16):
        for edge in (1008 * k, 1024 * k):
            for r in (1, 2, 3, 8, 9, 10, 11, 18, 19):
                for side in (-1, 0, 1):
                    n = min(16384, edge + 40)
                    x = bytearray(O.gen(1, 97 * edge + r, n))
                    lo = max(0, edge - r if side <= 0 else edge)
                    hi = min(n, edge + r if side >= 0 else edge)
                    x[lo:hi] = (b"7" if r % 2 else b"\0") * (hi - lo)
                    xs.append(bytes(x))
    rng = np.random.default_rng(17)
    for i in range(400):
        s = int(rng.integers(900, 16384))
        alpha = np.frombuffer(rng.choice([b"a0123456789", b"\0\x01", b"33", b"ab", b"99"]), np.uint8)
        xs.append(np.repeat(rng.choice(alpha, size=s), rng.integers(1, 22, size=s))[:s].tobytes())
    coop_parity(xs, dec_hints=(16128, 16384))


def test_golden_vectors(vectors):
    cases = [v for g in ("kat", "edge", "ladder", "fuzz") for v in vectors[g]]
    xs = [bytes.fromhex(v["in"]) for v in cases]
    ys = [bytes.fromhex(v["out"]) for v in cases]
    got, st = gpu_encode(xs, max_len=max(len(x) for x in xs))
    assert got == ys and (st == 0).all()
    dec, st = gpu_decode(ys, [len(x) for x in xs], max_in_len=max(len(y) for y in ys),
                         max_out_len=max(len(x) for x in xs))
    assert dec == xs and ((st & 0xFF) == 0).all()


def test_invalid_streams_and_overflow(vectors):
    # streams the tiled path declines take the exact serial decoder inside the cooperative kernel
    cases = vectors["invalid_decode"]
    streams = [bytes.fromhex(v["in"]) for v in cases]
    us = [v["U"] for v in cases]
    caps = [v["U"] + v["E"] for v in cases]
    dec, st = gpu_decode(streams, us, caps, poison=False, max_in_len=max(2048, max(len(s) for s in streams)),
                         max_out_len=max(us))
    bad = [i for i in range(len(cases)) if dec[i] != bytes.fromhex(cases[i]["out"])]
    assert not bad, (len(bad), cases[bad[0]], dec[bad[0]].hex())
    dec, st = gpu_decode([b"aa9" * 3, b"aa9", b"b" * 1500], [2, 9, 1500], [2, 9, 1500], max_in_len=1500,
                         max_out_len=1500)
    assert st[0] & 1 and dec[0] == b"aa" and st[1] == 0 and dec[1] == b"a" * 9 and dec[2] == b"b" * 1500


def test_hints_smaller_than_buffers_fall_back():
    # buffers past the kernel's tiles (or, decode, its staging) are walked by wave 0 alone
    xs = [O.gen(i % 5, 300 + i, s) for i, s in enumerate([3000, 9000, 20000, 70000, 1500, 100, 4096, 16385])]
    coop_parity(xs, enc_hint=2048, dec_hints=(2016, 4096))
    coop_parity(xs, enc_hint=8192, dec_hints=(8064, 16384))


@pytest.mark.parametrize("coop", [1, 0])
def test_completion_flag_launches_same_bytes(coop):
    """RLE_LAUNCH_STATUS_FLAG (include/rle_mi355x.h, the drop-in's polled small calls): the status is
    stored last behind a system-scope release; output, sizes and status are the same as without it,
    in the cooperative kernels (multi-wave release before the barrier) and the one-wave kernels,
    including their bad-slot, one-wave-fallback, short and serial exits."""
    import rle_mi355x as R
    R.set_coop_mode(coop)
    sizes = [0, 1, 17, 1008, 1009, 2049, 4096, 5000, 8192, 12000, 16384]
    xs = [O.gen(k % 5, 31 * k + 7, s) for k, s in enumerate(sizes)]
    refs = [O.encode(x) for x in xs]
    mx = max(len(x) for x in xs)
    for hint in (mx, 4096):   # 4096: the longer buffers take the workgroup's one-wave fallback
        ys, st = gpu_encode(xs, max_len=hint, flags=R.RLE_LAUNCH_STATUS_FLAG)
        assert ys == refs and (st == 0).all(), st
    streams = list(refs) + [b"aa:" + refs[4], b"abc", b"xx9" * 300]
    us = [len(x) for x in xs] + [len(xs[4]), 5, 3000]
    caps = list(us)
    caps[len(xs)] += 64
    mi = max(len(s) for s in streams)
    for hints in ((mi, max(us)), (2016, 4096)):
        got, st = gpu_decode(streams, us, caps, max_in_len=hints[0], max_out_len=hints[1],
                             flags=R.RLE_LAUNCH_STATUS_FLAG)
        ref, rst = gpu_decode(streams, us, caps, max_in_len=hints[0], max_out_len=hints[1])
        assert got == ref and (st == rst).all(), (st, rst)
        for i in range(len(xs)):
            assert got[i] == xs[i], i
        assert st[len(xs)] & R.RLE_STATUS_SERIAL and st[len(xs) + 1] == R.RLE_STATUS_SHORT
    R.set_coop_mode(1)


def test_worst_case_32k_streams_take_four_rounds():
    """a 16-32 KiB buffer whose stream is past 48 tiles (all runs of length 2: C = 1.5 U,
    up to 49152 bytes = 49 tiles) now takes the four-round workgroup (dec_coop_kernel<16, 32768, 4>)
    instead of the one-wave fallback; sizes around the 48-tile edge, bit-exact."""
    xs = []
    for U in (32768, 32767, 32256, 32254, 32250, 30000, 24000, 16385):
        xs.append(O.gen(4, U, U))   # kind 4: pairs (the 1.5x worst case)
    coop_parity(xs)
