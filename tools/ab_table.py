#!/usr/bin/env python3
"""Median codec kernel durations of tools/ab.sh runs: one row per (workload, kernel), one column per
library build.   usage: python tools/ab_table.py gpurun_out/<tag> [more tags...]"""
import collections
import csv
import glob
import os
import sys

res = collections.defaultdict(lambda: collections.defaultdict(list))
libs = []
for d in sys.argv[1:]:
    for path in glob.glob(os.path.join(d, "librle_*_*", "run_kernel_trace.csv")):
        tag = os.path.basename(os.path.dirname(path))
        lib = next(l for l in ("librle_mi355x",) + tuple(sorted({os.path.basename(p)[:-3] for p in glob.glob(
            os.path.join(os.environ.get("VARDIR", "c-filestorage-server-and-client_amd/build/variants"), "*.so"))}))
                   if tag.startswith(l + "_"))
        wl = tag[len(lib) + 1:]
        if lib not in libs:
            libs.append(lib)
        for r in csv.DictReader(open(path)):
            n = r["Kernel_Name"]
            if "encode_kernel" in n or "decode_kernel" in n:
                k = "enc" if "encode" in n else "dec"
                res[(wl, k)][lib].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
print(f"{'workload':12s} {'k':3s} " + " ".join(f"{l[7:]:>16s}" for l in libs))
for (wl, k), per in sorted(res.items()):
    cells = []
    for l in libs:
        v = sorted(per.get(l, []))
        cells.append(f"{v[len(v) // 2]:9.2f}/{v[0]:6.1f}" if v else " " * 16)
    print(f"{wl:12s} {k:3s} " + " ".join(cells))
