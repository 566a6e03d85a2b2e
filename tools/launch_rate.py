#!/usr/bin/env python3
"""Host enqueue rate of the bench step (encode + decode launch through rle_mi355x's ctypes
launchers) against the GPU time per step: if enqueueing a step takes longer than the GPU needs to
run it, the bench measures the host, not the kernels.
usage: python tools/launch_rate.py [--workload cfg1] [--steps 400]"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]
import torch  # noqa: E402

import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="cfg1")
ap.add_argument("--steps", type=int, default=400)
a = ap.parse_args()
dev = torch.device("cuda", 0)
B = bench.Batch(bench.WORKLOADS[a.workload], 0, 1, dev)
B.calibrate()
s = torch.cuda.current_stream()
for _ in range(20):
    B.encode(s)
    B.decode(s)
torch.cuda.synchronize()

t0 = time.perf_counter()
for _ in range(a.steps):
    B.encode(s)
    B.decode(s)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
enq = (t1 - t0) / a.steps * 1e6
tot = (t2 - t0) / a.steps * 1e6

# GPU-only time per step: events around the same loop after the queue has drained
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(s)
for _ in range(a.steps):
    B.encode(s)
    B.decode(s)
e1.record(s)
torch.cuda.synchronize()
gpu = e0.elapsed_time(e1) / a.steps * 1e3

# the same step captured once in a HIP graph and replayed
g = torch.cuda.CUDAGraph()
cs = torch.cuda.Stream()
cs.wait_stream(s)
with torch.cuda.stream(cs):
    with torch.cuda.graph(g, stream=cs):
        B.encode(cs)
        B.decode(cs)
torch.cuda.synchronize()
for _ in range(20):
    g.replay()
torch.cuda.synchronize()
t3 = time.perf_counter()
for _ in range(a.steps):
    g.replay()
t4 = time.perf_counter()
torch.cuda.synchronize()
t5 = time.perf_counter()
ok = B.verify() if hasattr(B, "verify") else None
print(f"{a.workload}: host enqueue {enq:.1f} us/step, wall {tot:.1f} us/step, GPU events {gpu:.1f} us/step; "
      f"graph replay: enqueue {(t4 - t3) / a.steps * 1e6:.1f} us/step, wall {(t5 - t3) / a.steps * 1e6:.1f} us/step; verify {ok}")
