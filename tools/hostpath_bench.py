#!/usr/bin/env python3
"""Host-path rate of the drop-in RLEcompress / RLEdecompress (BASELINE configs[4] component):
the rate a caller such as src/filesystemApi.c sees, starting and ending in host memory
(caller bytes -> pinned staging -> H2D -> kernel -> D2H -> fresh malloc block), for single
calls of various sizes and for T concurrent threads (the server's worker pool, src/server.c:520).

Prints one JSON object; the numbers feed DESIGN.md §6.
usage: python tools/hostpath_bench.py [--seconds 2]
"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "c-filestorage-server-and-client_amd")]
import rle_mi355x as R  # noqa: E402


def gen(kind, U, seed):
    import random
    rnd = random.Random(seed)
    if kind == "zero":
        return bytes(U)
    if kind == "random":
        return rnd.randbytes(U)
    out = bytearray()
    while len(out) < U:   # runs50-like
        out += bytes([rnd.randrange(256)]) * (1 + int(rnd.expovariate(1.0)))
    return bytes(out[:U])


def one(kind, U, seconds):
    L = R.lib()
    x = gen(kind, U, U)
    c = ctypes.c_size_t(0)
    # warm up (per-thread context, staging growth)
    p = L.RLEcompress(x, U, ctypes.byref(c))
    y = ctypes.string_at(p, c.value)
    R._libc.free(p)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        p = L.RLEcompress(x, U, ctypes.byref(c))
        R._libc.free(p)
        n += 1
    tc = (time.perf_counter() - t0) / n
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        p = L.RLEdecompress(y, len(y), U, 0)
        R._libc.free(p)
        n += 1
    td = (time.perf_counter() - t0) / n
    return {"kind": kind, "U": U, "C": len(y), "compress_us": tc * 1e6, "decompress_us": td * 1e6,
            "compress_GBps": U / tc / 1e9, "decompress_GBps": U / td / 1e9}


def threads(T, U, seconds):
    """T threads, each round-tripping its own U random bytes (the server's requests each have their
    own buffers, src/server.c:150-151)."""
    L = R.lib()
    xs = [gen("random", U, 7 + i) for i in range(T)]
    counts = [0] * T
    stop = time.perf_counter() + seconds

    def work(i):
        x = xs[i]
        c = ctypes.c_size_t(0)
        while time.perf_counter() < stop:
            p = L.RLEcompress(x, U, ctypes.byref(c))
            y = ctypes.string_at(p, c.value)
            R._libc.free(p)
            q = L.RLEdecompress(y, len(y), U, 0)
            R._libc.free(q)
            counts[i] += 1

    th = [threading.Thread(target=work, args=(i,)) for i in range(T)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    el = time.perf_counter() - t0
    return {"threads": T, "U": U, "roundtrips": sum(counts), "roundtrip_GBps": sum(counts) * U / el / 1e9}


def _timeit(fn, seconds):
    fn()
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        fn()
        n += 1
    return (time.perf_counter() - t0) / n


def write_path(L, x, new):
    """src/filesystemApi.c:767-775 through codec library L (decode with E extra, memcpy, encode)."""
    y_c = ctypes.c_size_t(0)
    U = len(x)

    def run(y, C):
        d = L.RLEdecompress(y, C, U, len(new))
        ctypes.memmove(d + U, new, len(new))
        p = L.RLEcompress(ctypes.cast(d, ctypes.c_char_p), U + len(new), ctypes.byref(y_c))
        R._libc.free(d)
        R._libc.free(p)
    return run


def fileops(seconds):
    """SURVEY §8 (f1) fused append vs the reference's three-call write path, and (f2)/(f4) one
    batched RLEdecompressN vs a loop of RLEdecompress calls (readNFiles / eviction)."""
    L = R.lib()
    L.RLEdecompress.restype = ctypes.c_void_p
    out = {"append": [], "readN": []}
    ref = None
    try:
        sys.path[:0] = [os.path.join(REPO, "oracle")]
        import rle_oracle as O
        ref = O.reference()   # the compiled reference codec (oracle/_ref), CPU, one thread
    except Exception:
        O = None
    for kind, U, A in (("random", 4096, 4096), ("runs", 65536, 4096), ("random", 1 << 20, 4096),
                       ("zero", 4 << 20, 65536), ("runs", 4 << 20, 65536)):
        x, new = gen(kind, U, 3), gen(kind, A, 4)
        y = R.compress(x)
        C = len(y)
        c = ctypes.c_size_t(0)

        def fused():
            p = L.RLEappend(y, C, U, new, A, ctypes.byref(c))
            R._libc.free(p)
        t_f = _timeit(fused, seconds)
        t_c = _timeit(lambda: write_path(L, x, new)(y, C), seconds)
        row = {"kind": kind, "U": U, "A": A, "C": C, "fused_us": t_f * 1e6, "composed_gpu_us": t_c * 1e6}
        if ref is not None:
            ypad = y + b"\0\0\0"
            t_r = _timeit(lambda: write_path(ref, x, new)(ypad, C), min(seconds, 2.0))
            row["reference_cpu_us"] = t_r * 1e6
        out["append"].append(row)
        print(f"append {kind} {U} done", file=sys.stderr, flush=True)
    # uniform batches, then a mixed one: 255 small files and one of 1 MiB (segmented + one-wave)
    for n, U in ((64, 4096), (256, 4096), (64, 65536), (16, 1 << 20), (256, None)):
        Us = [U] * n if U else [4096] * (n - 1) + [1 << 20]
        xs = [gen(("random", "zero", "runs")[i % 3], Us[i], i) for i in range(n)]
        ys = [R.compress(x) for x in xs]
        bufs = [ctypes.create_string_buffer(Us[k]) for k in range(n)]
        keep = [ctypes.create_string_buffer(y, len(y) + 3) for y in ys]
        data = (ctypes.c_void_p * n)(*[ctypes.addressof(k) for k in keep])
        cs = (ctypes.c_size_t * n)(*[len(y) for y in ys])
        us = (ctypes.c_size_t * n)(*Us)
        op = (ctypes.c_void_p * n)(*[ctypes.addressof(b) for b in bufs])

        def batched():
            assert L.RLEdecompressN(n, data, cs, us, op) == 0

        def looped():
            for k in range(n):
                p = L.RLEdecompress(keep[k], cs[k], Us[k], 0)
                ctypes.memmove(bufs[k], p, Us[k])
                R._libc.free(p)
        t_b = _timeit(batched, seconds)
        t_l = _timeit(looped, seconds)
        assert all(bufs[k].raw == xs[k] for k in range(n))
        tot = sum(Us)
        out["readN"].append({"files": n, "U": U or "255 x 4 KiB + 1 MiB", "batched_us": t_b * 1e6,
                             "looped_us": t_l * 1e6, "batched_GBps": tot / t_b / 1e9, "looped_GBps": tot / t_l / 1e9})
        print(f"readN {n}x{U} done", file=sys.stderr, flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=1.0)
    ap.add_argument("--only", choices=["single", "threads", "fileops"], default=None)
    ap.add_argument("--sizes", default="4096,65536,1048576,4194304", help="single-call sizes, bytes")
    a = ap.parse_args()
    R.dropin_stats(reset=True)
    res = {"single": [], "threads": []}
    if a.only in (None, "single"):
        for U in (int(v) for v in a.sizes.split(",")):
            for kind in ("random", "zero", "runs"):
                res["single"].append(one(kind, U, a.seconds))
    if a.only in (None, "fileops"):
        res["fileops"] = fileops(a.seconds)
    if a.only in (None, "threads"):
        for T in (1, 4, 8):
            res["threads"].append(threads(T, 1 << 20, a.seconds))
            print(f"threads {T} done", file=sys.stderr, flush=True)
    s = R.dropin_stats()
    res["dropin_stats"] = s
    tot = s["ns_stage_in"] + s["ns_device"] + s["ns_stage_out"]
    res["phase_share"] = {k: s[k] / tot for k in ("ns_stage_in", "ns_device", "ns_stage_out")} if tot else None
    res["pcie_GBps_device_phase"] = (s["bytes_h2d"] + s["bytes_d2h"]) / (s["ns_device"] * 1e-9) / 1e9 \
        if s["ns_device"] else None
    print(json.dumps(res), flush=True)
    print("main done", file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
