#!/usr/bin/env python3
"""Throughput of configs[1] round trips issued on one stream vs on two or four streams (each stream
with its own batch buffers), to see how much independent launches overlapping on the GPU gain
over back-to-back launches.  usage: python tools/overlap_probe.py [--workload cfg1] [--steps 200]"""
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
ap.add_argument("--steps", type=int, default=200)
a = ap.parse_args()
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
wl = bench.WORKLOADS[a.workload]
for nstreams in (1, 2, 4):
    Bs = [bench.Batch(wl, 0, 1, dev) for _ in range(nstreams)]
    ss = [torch.cuda.Stream(device=dev) for _ in range(nstreams)]
    for B, s in zip(Bs, ss):
        B.encode(s)
        B.calibrate()
    for _ in range(3):
        for B, s in zip(Bs, ss):
            B.encode(s)
            B.decode(s)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(a.steps):
        B, s = Bs[k % nstreams], ss[k % nstreams]
        B.encode(s)
        B.decode(s)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ok = all(torch.equal(B.d_out, B.d_in) for B in Bs)
    print(f"{a.workload} streams={nstreams}: {dt / a.steps * 1e6:.2f} us per round trip, "
          f"{Bs[0].u_bytes * a.steps / dt / 2**30:.1f} GiB/s, ok={ok}")
    del Bs
    torch.cuda.empty_cache()
