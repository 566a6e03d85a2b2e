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
    L = R.lib()
    x = gen("random", U, 7)
    counts = [0] * T
    stop = time.perf_counter() + seconds

    def work(i):
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=1.0)
    ap.add_argument("--only", choices=["single", "threads"], default=None)
    a = ap.parse_args()
    R.dropin_stats(reset=True)
    res = {"single": [], "threads": []}
    if a.only != "threads":
        for U in (4096, 65536, 1 << 20, 4 << 20):
            for kind in ("random", "zero", "runs"):
                res["single"].append(one(kind, U, a.seconds))
    if a.only != "single":
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
