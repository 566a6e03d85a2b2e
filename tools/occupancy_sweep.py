#!/usr/bin/env python3
"""Latency or throughput?  Times encode / decode of n x 4 KiB buffers of one kind for n from 256
(one wave per SIMD, or fewer) to 16384 (four residency rounds), HIP events around `reps`
back-to-back launches.  A launch whose time stays flat as n grows is bound by each wave's own
chain; one whose time grows with n is bound by what the SIMDs share (issue, LDS, memory).
usage: python tools/occupancy_sweep.py [--reps 20] [--size 4096] [--coop 0]"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]
import torch  # noqa: E402

import bench  # noqa: E402
import rle_mi355x as R  # noqa: E402


def timed(fn, reps, s):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = None
    for _ in range(3):
        e0.record(s)
        for _ in range(reps):
            fn()
        e1.record(s)
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) * 1e3 / reps
        best = t if best is None else min(best, t)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--coop", type=int, default=0, help="cooperative small-buffer kernels: 0 never (one wave per buffer), -1 the default")
    a = ap.parse_args()
    R.set_coop_mode(a.coop)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    s = torch.cuda.current_stream()
    rows = []
    for kind, name in ((1, "random"), (0, "zero"), (2, "runs50")):
        for n in (256, 512, 1024, 2048, 4096, 8192, 16384):
            B = bench.Batch(dict(n=n, size=a.size, kinds=(kind,)), 0, 1, dev)
            B.encode(s)
            B.calibrate()
            te = timed(lambda: B.encode(s), a.reps, s)
            td = timed(lambda: B.decode(s), a.reps, s)
            ok = B.verify()
            row = {"kind": name, "n": n, "enc_us": round(te, 2), "dec_us": round(td, 2),
                   "waves_per_simd": round(n / 1024, 2), "ok": ok}
            rows.append(row)
            print(json.dumps(row), flush=True)
            del B
            torch.cuda.empty_cache()
    print(json.dumps({"rows": rows}))


if __name__ == "__main__":
    main()
