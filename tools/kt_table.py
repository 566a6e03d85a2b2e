#!/usr/bin/env python3
"""Median kernel durations per workload from rocprofv3 --kernel-trace runs of tools/prof_driver.py
(gpurun_out/<tag>/kt_<workload>/run_kernel_trace.csv).   usage: python tools/kt_table.py <dir>"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
for path in sorted(glob.glob(os.path.join(d, "kt_*", "run_kernel_trace.csv"))):
    wl = os.path.basename(os.path.dirname(path))[3:]
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if "encode" in name or "decode" in name or "dec_order" in name:
            key = name.split("(")[0].replace("void ", "").replace("rle::", "")
            dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
    for k, v in sorted(dur.items()):
        v.sort()
        print(f"{wl:12s} {k:32s} n={len(v):2d} median={v[len(v) // 2]:9.2f} us  min={v[0]:9.2f}")
