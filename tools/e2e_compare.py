#!/usr/bin/env python3
"""Side-by-side wall times of the UNCHANGED reference server linked against the reference codec
(server_ref, BASELINE configs[0]) and against librle_mi355x.so (server_gpu, configs[4]), on the
batteries of tests/test_e2e_server.py plus a concurrent one:

  battery1   tests/test1.sh:13,17 flows (1 worker): write file1,file2, read back; write rec/, read all
  battery2   tests/test2.sh:6-30 LRU eviction (4 workers), evicted file decoded and shipped back
  battery3   8 clients at once (8 workers; the tests/test3.sh shape): a cold round (one small file
             each, on a fresh server), then each writes its own 64 small files (4-40 KiB, random /
             zero / runs) with -w and reads them back one by one with -r, so the codec sees
             concurrent small compress and decompress calls on warm worker threads

Batteries 1 and 2 are timed twice: from the moment the server's socket appears (cold: the first
calls may still wait for the drop-in's background start-up) and on a server that has been up for
SETTLE seconds (started: a serving process).  Every returned file is checked byte for byte.
startup_s: spawn to socket (battery 3's server; the drop-in's start-up phase 1 runs before main()
since round 5).  server_gpu also runs with RLE_MI355X_PREINIT_WAIT_MS=0 (round 4: the start-up in
the background only), RLE_MI355X_PREINIT=0 (round 3's lazy start-up on the first call) and with
RLE_MI355X_ZC_SEG=0 (no zero-copy segmented form: round 4's first form of the small calls).
Prints one JSON object.   usage: python tools/e2e_compare.py [--reps 3]
"""
import argparse
import json
import os
import random
import shutil
import sys
import tempfile
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests")]
import test_e2e_server as E  # noqa: E402


def make_files(tmp, c, nfiles, rnd):
    d = os.path.join(tmp, f"c{c}")
    os.makedirs(d, exist_ok=True)
    files = {}
    for k in range(nfiles):
        U = rnd.choice([4096, 8192, 16384, 40000])
        kind = k % 3
        b = bytes(U) if kind == 1 else (rnd.randbytes(U) if kind == 0 else
                                        b"".join(bytes([rnd.randrange(256)]) * rnd.randrange(1, 12)
                                                 for _ in range(U // 4))[:U])
        p = os.path.join(d, f"f{c}_{k}")
        with open(p, "wb") as f:
            f.write(b)
        files[p] = b
    return d, files


def concurrent_round(srv, tmp, dirs, tag):
    """Each client c writes its directory (-w) and reads its files back one by one (-r)."""
    errs = []

    def client(c, d, names):
        try:
            srv.client("-w", f"{d},0")
            srv.client("-r", ",".join(names), "-d", os.path.join(tmp, f"{tag}_out{c}"))
        except Exception as e:
            errs.append(repr(e))

    t0 = time.perf_counter()
    th = [threading.Thread(target=client, args=(c, d, sorted(fs))) for c, (d, fs) in enumerate(dirs)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    wall = time.perf_counter() - t0
    assert not errs, errs[:3]
    return wall


def battery3(exe, tmp, env=None):
    """8 workers, 8 concurrent clients.  cold: a fresh server's first round (1 small file per client:
    for server_gpu that includes HIP runtime start-up and the 8 worker threads' codec contexts);
    warm: the same server, then 64 files per client."""
    rnd = random.Random(3)
    warm = [make_files(os.path.join(tmp, "warm"), c, 1, rnd) for c in range(8)]
    main = [make_files(os.path.join(tmp, "main"), c, 64, rnd) for c in range(8)]
    srv = E.Server(exe, tmp, {"MAXSTORAGECAP": 512000000, "MAXFILECOUNT": 10000, "WORKERPOOLSIZE": 8}, env)
    try:
        cold = concurrent_round(srv, tmp, warm, "warm")
        hot = concurrent_round(srv, tmp, main, "main")
    finally:
        srv.stop()
    battery3.startup_s = srv.startup_s
    got = E._returned(tmp)
    for d, fs in warm + main:
        for p, b in fs.items():
            assert b in got.get(os.path.basename(p), []), p
    return cold, hot


SETTLE = 1.5


def run(exe, env, reps):
    out = {"battery1_s": [], "battery1_started_s": [], "battery2_s": [], "battery2_started_s": [],
           "battery3_cold_s": [], "battery3_warm_s": [], "startup_s": []}
    for _ in range(reps):
        for settle, key in ((0.0, ""), (SETTLE, "_started")):
            with tempfile.TemporaryDirectory() as tmp:
                r1 = E.battery1(exe, os.path.join(tmp, "b1"), env, settle)
                E._check_battery1(r1)
                out["battery1%s_s" % key].append(round(r1[3], 4))
            with tempfile.TemporaryDirectory() as tmp:
                r2 = E.battery2(exe, os.path.join(tmp, "b2"), env, settle)
                E._check_battery2(r2)
                out["battery2%s_s" % key].append(round(r2[3], 4))   # from the socket's appearance, less the sleep
        with tempfile.TemporaryDirectory() as tmp:
            cold, hot = battery3(exe, tmp, env)
            out["battery3_cold_s"].append(round(cold, 4))
            out["battery3_warm_s"].append(round(hot, 4))
            out["startup_s"].append(round(battery3.startup_s, 4))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    res = {}
    for name, exe, env in (("server_ref", "server_ref", None),
                           ("server_gpu", "server_gpu", None),
                           ("server_gpu_nowait", "server_gpu", {"RLE_MI355X_PREINIT_WAIT_MS": "0"}),
                           ("server_gpu_preinit0", "server_gpu", {"RLE_MI355X_PREINIT": "0"}),
                           ("server_gpu_zcseg0", "server_gpu", {"RLE_MI355X_ZC_SEG": "0"})):
        path = os.path.join(E.BIN, exe)
        if not os.path.exists(path):
            res[name] = "not built"
            continue
        res[name] = run(path, env, a.reps)
        print(name, "done", file=sys.stderr, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
