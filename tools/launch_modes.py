#!/usr/bin/env python3
"""Why do HIP events around back-to-back launches (tools/ab_events.py, bench.py's time_kernels) and
rocprofv3's per-dispatch kernel durations disagree for some 64 KiB kinds (r4a: runs50 decode 532 us
against 659 us on one box)?  Times each codec call of a workload three ways in one process:
  single    synchronize, event, one call, event, synchronize (per call)
  b2b       events around `reps` calls issued back to back, divided by reps
  b2b_sync  the same `reps` calls with a stream synchronize after each, host wall / reps
Prints one JSON object per workload.   usage: python tools/launch_modes.py [--workloads k64_runs50] [--reps 10]"""
import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="k64_runs50,k64_runs90,k64_random,k64_zero,dec64k,cfg1")
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    s = torch.cuda.current_stream()
    for wl in a.workloads.split(","):
        B = bench.Batch(bench.WORKLOADS[wl], 0, 1, dev)
        B.encode(s)
        B.calibrate()
        out = {"workload": wl}
        for name, fn in (("encode", lambda: B.encode(s)), ("decode", lambda: B.decode(s))):
            fn()
            torch.cuda.synchronize()
            single = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record(s)
                fn()
                e1.record(s)
                torch.cuda.synchronize()
                single.append(e0.elapsed_time(e1) * 1e3)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(a.reps):
                fn()
            e1.record(s)
            torch.cuda.synchronize()
            b2b = e0.elapsed_time(e1) * 1e3 / a.reps
            t0 = time.perf_counter()
            for _ in range(a.reps):
                fn()
                torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) * 1e6 / a.reps
            out[name] = {"single_median_us": round(statistics.median(single), 1), "single_min_us": round(min(single), 1),
                         "b2b_us": round(b2b, 1), "b2b_sync_wall_us": round(wall, 1)}
        out["roundtrip_ok"] = bool(torch.equal(B.d_out, B.d_in))
        print(json.dumps(out), flush=True)
        del B
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
