#!/usr/bin/env python3
"""Where a short timed bench region loses time: after bench.py's own warmup (W steps and the
verification), per-step durations of the next K steps from HIP events on the launch stream, and the
host wall time of the whole region (the bench's clock).  usage: python tools/step_profile.py [--steps 20] [--warmup 5]"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]
import torch  # noqa: E402

import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--warmup", type=int, default=5)
ap.add_argument("--bench-order", action="store_true",
                help="as bench.py: verify (host work, GPU idle) first, then the W warmup steps, then time")
a = ap.parse_args()
dev = torch.device("cuda", 0)
s = torch.cuda.current_stream()
B = bench.Batch(bench.WORKLOADS["cfg1"], 0, 1, dev)
B.encode(s)
B.calibrate()
if a.bench_order:
    B.encode(s)
    B.decode(s)
    torch.cuda.synchronize()
    ok = bool(torch.equal(B.d_out, B.d_in)) and int(B.status.abs().sum().item()) == 0
    _ = int(B.clen.sum().item())
for _ in range(a.warmup):
    B.encode(s)
    B.decode(s)
torch.cuda.synchronize()
if not a.bench_order:
    ok = bool(torch.equal(B.d_out, B.d_in))
for rnd in range(3):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev[0].record(s)
    for k in range(a.steps):
        B.encode(s)
        B.decode(s)
        ev[k + 1].record(s)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e6
    d = [ev[k].elapsed_time(ev[k + 1]) * 1e3 for k in range(a.steps)]
    print(f"round {rnd}: wall {wall:.1f} us = {wall / a.steps:.2f} us/step; events sum {sum(d):.1f} us; "
          f"per step: {' '.join(f'{x:.1f}' for x in d)}; verified {ok}")
