#!/usr/bin/env python3
"""Profiling driver: build one bench workload in HBM and run encode / decode launches only,
so rocprofv3 traces and PMC passes see the codec kernels without the generator or checks.
--warm W: W encodes and W decodes first (untimed: the shader clock ramps over the first ~10 ms of
run-heavy work, profiles/r5al_pattern_rounds.jsonl); then --rounds rounds of --reps encodes and
--reps decodes (the bench's steady-state timing; tools/kinds_table.py --skip W + 1 drops the warm
launches and the calibration encode).
usage: python tools/prof_driver.py [--workload dec64k] [--reps 5] [--warm 0] [--rounds 1]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]
import torch  # noqa: E402

import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="dec64k")
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--warm", type=int, default=0)
ap.add_argument("--rounds", type=int, default=1)
ap.add_argument("--seg", action="store_true", help="segmented (several waves per buffer) entry points")
a = ap.parse_args()
torch.cuda.set_device(0)
B = bench.Batch(bench.WORKLOADS[a.workload], 0, 1, torch.device("cuda", 0))
B.seg = a.seg
s = torch.cuda.current_stream()
B.encode(s)
B.calibrate()
for _ in range(a.warm):
    B.encode(s)
for _ in range(a.warm):
    B.decode(s)
for _ in range(a.rounds):
    for _ in range(a.reps):
        B.encode(s)
    for _ in range(a.reps):
        B.decode(s)
torch.cuda.synchronize()
ok = torch.equal(B.d_out, B.d_in)
print("ok" if ok else "MISMATCH", B.u_bytes, int(B.clen.sum().item()))
sys.exit(0 if ok else 1)
