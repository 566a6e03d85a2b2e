"""CPU tests: the oracle (oracle/rle_oracle.c) pinned against the golden vectors produced by the
compiled reference (tests/golden/make_golden.py), the report's KAT and the reference fixture pins
(SURVEY.md Appendix B); plus a live cross-check against oracle/_ref when it is built here."""
import hashlib
import os
import random

import pytest

import rle_oracle as O
from conftest import committed_file_bytes


def sha(b):
    return hashlib.sha256(b).hexdigest()


def test_kat_relazione():
    # Relazione.pdf p.3 "Compressione": aaaaaaaaaaaab -> aa9aa3b
    assert O.encode(b"aaaaaaaaaaaab") == b"aa9aa3b"
    assert O.decode(b"aa9aa3b", 13)[0] == b"aaaaaaaaaaaab"


@pytest.mark.parametrize("group", ["kat", "edge", "ladder", "fuzz"])
def test_encode_golden(vectors, group):
    for v in vectors[group]:
        x, y = bytes.fromhex(v["in"]), bytes.fromhex(v["out"])
        assert O.encode(x) == y, v
        out, st = O.decode(y, len(x))
        assert st == 0 and out == x, v


def test_ladder_closed_form(vectors):
    # per-run size 3*floor((L-1)/9) + (3 if (L-1)%9 else 1)  
    for v in vectors["ladder"]:
        L = len(bytes.fromhex(v["in"]))
        assert len(bytes.fromhex(v["out"])) == 3 * ((L - 1) // 9) + (3 if (L - 1) % 9 else 1)


def test_synthetic_pins(vectors):
    for v in vectors["synthetic"]:
        if v["U"] > 70000:
            continue
        x = O.gen(v["kind"], v["index"], v["U"])
        assert sha(x) == v["sha_in"], v
        y = O.encode(x)
        assert len(y) == v["C"] and sha(y) == v["sha_out"], v
        assert O.decode(y, len(x))[0] == x


def test_synthetic_pins_1mib(vectors):
    for v in vectors["synthetic"]:
        if v["U"] <= 70000:
            continue
        x = O.gen(v["kind"], v["index"], v["U"])
        y = O.encode(x)
        assert sha(x) == v["sha_in"] and len(y) == v["C"] and sha(y) == v["sha_out"], v


def test_invalid_stream_decode(vectors):
    # streams the encoder never emits: reference output of U+E bytes pinned
    for v in vectors["invalid_decode"]:
        y = bytes.fromhex(v["in"])
        out, st = O.decode(y, v["U"], v["U"] + v["E"])
        assert st == 0 and out == bytes.fromhex(v["out"]), v


def test_decode_overflow_is_reported():
    # "aa9" x 3 decodes to 27 bytes; with U = 2 and no E the reference writes past its block
    out, st = O.decode(b"aa9" * 3, 2, 2)
    assert st == 1 and out == b"aa"


def test_reference_fixture_pins(dummyfiles):
    n = 0
    for e in dummyfiles["files"]:
        x = committed_file_bytes(e)
        if x is None:
            continue
        assert sha(x) == e["sha_in"]
        y = O.encode(x)
        assert len(y) == e["C"] and sha(y) == e["sha_out"], e["path"]
        assert O.decode(y, len(x))[0] == x
        n += 1
    assert n >= 8


def test_test2_storage_statistic(dummyfiles):
    # tests/test2.sh: "Max total storage size reached: 942363 bytes" = C(big2) + C(randbig)
    by = {e["path"]: e for e in dummyfiles["files"]}
    assert by["bigfiles/big2"]["C"] + by["bigfiles/randbig"]["C"] == 942363
    assert dummyfiles["test2_max_storage"] == 942363
    assert len(O.encode(bytes(360000))) == by["bigfiles/big2"]["C"]


@pytest.mark.skipif(not os.path.exists(O.REF_SO), reason="oracle/_ref not built (needs /root/reference)")
def test_oracle_vs_compiled_reference_fuzz():
    rng = random.Random(7)
    for k in range(2000):
        L = rng.randint(0, 300)
        alpha = rng.choice([b"ab", b"a0123456789", b"\0\x01", bytes(range(256))])
        x = bytes(rng.choice(alpha) for _ in range(L))
        y = O.ref_compress(x)
        assert O.encode(x) == y
        for U in (len(x), max(0, len(x) - 3)):
            E = len(y) + 8
            assert O.decode(y, U, U + E)[0] == O.ref_decompress(y, U, E)
    for k in range(500):  # arbitrary streams
        L = rng.randint(1, 30)
        y = bytes(rng.choice(b"aa0123456789:/\0\x80\xff~") for _ in range(L))
        U = rng.randint(0, 60)
        E = L + 8
        assert O.decode(y, U, U + E)[0] == O.ref_decompress(y, U, E), (y, U)


def test_generator_kinds():
    assert O.gen(0, 5, 100) == bytes(100)
    p = O.gen(4, 9, 1000)
    y = O.encode(p)
    assert len(y) == 1500  # all runs of length 2
    r50 = O.gen(2, 1, 65536)
    assert 0.9 < len(O.encode(r50)) / 65536 < 1.1
    r90 = O.gen(3, 1, 65536)
    assert 0.35 < len(O.encode(r90)) / 65536 < 0.6
