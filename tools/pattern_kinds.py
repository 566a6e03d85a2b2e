#!/usr/bin/env python3
"""Decode against its memory-pattern ceiling per 64 KiB data kind (GPU box).

For each workload: the batched decode's launch time, rle_decode_pattern_device's (the same tile reads
and output writes, one wave per buffer, no token work) and the device copy of the same bytes, all as
GB/s of (U + C) and as fractions of 8 TB/s.  Prints one JSON object per workload.
  usage: python tools/pattern_kinds.py [--workloads k64_zero,k64_random,...] [--reps 20]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import torch  # noqa: E402

R = bench.R


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="k64_zero,k64_random,k64_runs50,k64_runs90,k64_z50,dec64k")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=1, help="timings per launch kind (the median is reported)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)
    for name in a.workloads.split(","):
        B = bench.Batch(bench.WORKLOADS[name], 0, 1, dev)
        B.encode(stream)
        B.calibrate()
        nc = int(B.clen.sum().item())
        alg = B.u_bytes + nc
        dec = lambda: B.decode(stream)
        pat = lambda: R.decode_pattern(B.d_c, B.coffs, B.clen, B.d_out, B.offs, B.lens, stream)
        tds = [bench.time_kernels(dec, a.reps, stream)]
        ok = bool(torch.equal(B.d_out, B.d_in))
        tps = []
        for r in range(a.rounds):   # alternating, so both see the same clocks
            tps.append(bench.time_kernels(pat, a.reps, stream))
            if r + 1 < a.rounds:
                tds.append(bench.time_kernels(dec, a.reps, stream))
        td, tp = sorted(tds)[len(tds) // 2], sorted(tps)[len(tps) // 2]
        cp = bench.copy_ceiling(B, alg, a.reps, stream)
        gb = lambda t: alg / t / 1e9
        print(json.dumps({"workload": name, "u_over_c": round(B.u_bytes / nc, 3), "verified": ok,
                          "decode_us": round(td * 1e6, 2), "decode_frac": round(gb(td) / 8000, 4),
                          "pattern_us": round(tp * 1e6, 2), "pattern_frac": round(gb(tp) / 8000, 4),
                          "copy_frac": cp["frac"], "decode_of_pattern": round(tp / td, 4),
                          "decode_us_rounds": [round(t * 1e6, 1) for t in tds],
                          "pattern_us_rounds": [round(t * 1e6, 1) for t in tps]}), flush=True)
        del B
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
