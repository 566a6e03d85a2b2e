#!/usr/bin/env python3
"""Generate the committed golden vectors from the COMPILED REFERENCE codec.

Runs only in the build container (needs /root/reference and `make -C oracle ref`):
it loads oracle/_ref/librle_ref_O0.so — /root/reference/src/rleCompression.c compiled
unchanged with the reference's own flags (Makefile:6) — and records its outputs.
Nothing here is shipped; the JSON/bin files it writes are data fixtures.

Outputs (tests/golden/):
  vectors.json      KAT, ladders, edge cases, fuzz (hex in/out), seeded synthetic pins
                    (sha256 of input and of compressed output), invalid-stream decodes
  dummyfiles.json   U, C, sha256 pins of every file in the reference's tests/dummyFiles
  dummyFiles/…      a few small fixture files copied as data (inputs of the reference's tests)
"""
import ctypes
import hashlib
import json
import os
import random
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_SO = os.path.join(REPO, "oracle", "_ref", "librle_ref_O0.so")
ORACLE_SO = os.path.join(REPO, "oracle", "librle_oracle.so")
REF_FILES = "/root/reference/tests/dummyFiles"

libc = ctypes.CDLL("libc.so.6")
libc.free.argtypes = [ctypes.c_void_p]


def load_ref():
    ref = ctypes.CDLL(REF_SO)
    ref.RLEcompress.restype = ctypes.c_void_p
    ref.RLEcompress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
    ref.RLEdecompress.restype = ctypes.c_void_p
    ref.RLEdecompress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t]
    return ref


REF = load_ref()
ORC = ctypes.CDLL(ORACLE_SO)
ORC.oracle_gen_buffer.argtypes = [ctypes.c_uint32, ctypes.c_uint64, ctypes.c_char_p, ctypes.c_size_t]


def ref_compress(data: bytes) -> bytes:
    c = ctypes.c_size_t(0)
    p = REF.RLEcompress(data, len(data), ctypes.byref(c))
    out = ctypes.string_at(p, c.value) if c.value else b""
    libc.free(p)
    return out


def ref_decompress(stream: bytes, U: int, E: int = 0) -> bytes:
    # the reference reads up to 2 bytes past C: hand it a zero-padded copy (its calloc padding)
    padded = stream + b"\0\0\0"
    p = REF.RLEdecompress(padded, len(stream), U, E)
    out = ctypes.string_at(p, U + E) if U + E else b""
    libc.free(p)
    return out


def gen(kind: int, index: int, U: int) -> bytes:
    buf = ctypes.create_string_buffer(max(U, 1))
    ORC.oracle_gen_buffer(kind, index, buf, U)
    return buf.raw[:U]


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def main():
    rng = random.Random(20261015)
    V = {"source": "reference src/rleCompression.c compiled unchanged (-Wall -g -std=c99)",
         "kat": [], "edge": [], "ladder": [], "fuzz": [], "synthetic": [], "invalid_decode": []}

    # KAT from Relazione.pdf p.3
    kat_in = b"aaaaaaaaaaaab"
    kat_out = ref_compress(kat_in)
    assert kat_out == b"aa9aa3b", kat_out
    V["kat"].append({"in": kat_in.hex(), "out": kat_out.hex()})

    edge = [b"", b"\0", b"\0\0", b"\0\0\0", b"a", b"ab", b"aa", b"aa2", b"aa222", b"333", b"3", b"33",
            b"aab", b"abb", b"abab", b"00", b"000", b"9" * 10, b"9" * 19, b"\xff" * 9, b"\xff" * 10,
            b"\x80\x80", b"a" * 1000, b"ab" * 500, b"\0" * 4096, b"\0" * 4097, b"\0" * 4095,
            b"x" + b"\0", b"xy\0", b"aa\0", b"\0" * 10 + b"a", b"a" + b"\0" * 10]
    for e in edge:
        c = ref_compress(e)
        assert ref_decompress(c, len(e)) == e
        V["edge"].append({"in": e.hex(), "out": c.hex()})

    for byte in (b"z", b"\0", b"0", b"9", b"\xff", b"\x80"):
        for L in range(1, 41):
            x = byte * L
            V["ladder"].append({"in": x.hex(), "out": ref_compress(x).hex()})

    # fuzz over small alphabets (digits and repeats are where decode alignment is subtle)
    alphabets = [b"ab", b"a0123456789", b"\0\x01", b"abc\0", bytes(range(256)), b"3", b"23"]
    for k in range(3000):
        alpha = alphabets[k % len(alphabets)]
        L = rng.randint(0, 96)
        mode = rng.random()
        if mode < 0.5:
            x = bytes(rng.choice(alpha) for _ in range(L))
        else:  # runs of random length
            out = bytearray()
            while len(out) < L:
                out += bytes([rng.choice(alpha)]) * rng.randint(1, 25)
            x = bytes(out[:L])
        c = ref_compress(x)
        assert ref_decompress(c, len(x)) == x
        V["fuzz"].append({"in": x.hex(), "out": c.hex()})

    # seeded synthetic buffers: pins of the generator and of the compressed output
    sizes = [1, 2, 3, 15, 16, 17, 63, 64, 65, 1023, 1024, 1025, 1039, 4095, 4096, 4097, 16384, 65536, 65537]
    for kind in range(5):
        for U in sizes:
            for index in (0, 1, 77):
                x = gen(kind, index, U)
                c = ref_compress(x)
                V["synthetic"].append({"kind": kind, "index": index, "U": U, "C": len(c),
                                       "sha_in": sha(x), "sha_out": sha(c)})
    for kind in range(5):
        x = gen(kind, 3, 1 << 20)
        c = ref_compress(x)
        V["synthetic"].append({"kind": kind, "index": 3, "U": 1 << 20, "C": len(c),
                               "sha_in": sha(x), "sha_out": sha(c)})

    # decodes of streams the encoder never emits: where the reference is well defined
    # (E large enough that nothing is written past U+E) its output U+E bytes are pinned.
    invalid = [b"aa0", b"aa1", b"aa:", b"aaA", b"aa/", b"aa\x80", b"aa\xff", b"aa", b"a", b"aaa",
               b"aa9aa", b"ab\0", b"\0", b"\0\0", b"\0\0\0", b"aa5bb5cc5", b"aa9" * 4, b"aaO",
               b"aa2bb", b"aa~xyz", b"xx\x7f", b"aa3bb3", b"zz9zz9zz9zz9"]
    for k in range(400):
        L = rng.randint(1, 40)
        invalid.append(bytes(rng.choice(b"aa0123456789:/\0\x80\xff") for _ in range(L)))
    for s in invalid:
        for U in sorted({0, 1, 2, 5, len(s), 3 * len(s), 9 * len(s)}):
            E = len(s) + 16  # every token writes at most 1 byte past U
            out = ref_decompress(s, U, E)
            V["invalid_decode"].append({"in": s.hex(), "U": U, "E": E, "out": out.hex()})

    with open(os.path.join(HERE, "vectors.json"), "w") as f:
        json.dump(V, f, separators=(",", ":"))

    # reference fixture files
    D = {"files": []}
    os.makedirs(os.path.join(HERE, "dummyFiles"), exist_ok=True)
    keep = {"file1", "file2", "rec/rec1", "rec/rec2", "smallfiles/small1", "smallfiles/small7", "bigfiles/randbig"}
    for root, _, files in os.walk(REF_FILES):
        for fn in sorted(files):
            p = os.path.join(root, fn)
            rel = os.path.relpath(p, REF_FILES)
            x = open(p, "rb").read()
            c = ref_compress(x)
            assert ref_decompress(c, len(x)) == x
            entry = {"path": rel, "U": len(x), "C": len(c), "sha_in": sha(x), "sha_out": sha(c),
                     "all_zero": x.count(0) == len(x), "committed": rel in keep}
            D["files"].append(entry)
            if rel in keep:
                dst = os.path.join(HERE, "dummyFiles", rel.replace("/", "__"))
                shutil.copyfile(p, dst)
                os.chmod(dst, 0o644)
    D["files"].sort(key=lambda e: e["path"])
    by = {e["path"]: e for e in D["files"]}
    D["test2_max_storage"] = by["bigfiles/big2"]["C"] + by["bigfiles/randbig"]["C"]
    with open(os.path.join(HERE, "dummyfiles.json"), "w") as f:
        json.dump(D, f, indent=1)
    print("vectors:", {k: len(v) for k, v in V.items() if isinstance(v, list)},
          "files:", len(D["files"]), "test2:", D["test2_max_storage"])


if __name__ == "__main__":
    sys.exit(main())
