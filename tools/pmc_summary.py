#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (one dir per pass) per codec kernel: mean counter value per
dispatch, and derived per-dispatch figures.  usage: python tools/pmc_summary.py gpurun_out/pmc_v2"""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "rle::" not in k:
            continue
        name = k.split("(")[0].replace("rle::", "")
        vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
out = {}
for k, d in vals.items():
    m = {c: sum(v) / len(v) for c, v in d.items()}
    out[k] = m
    print(f"== {k}: dispatches={len(d[next(iter(d))])}  mean dur(profiled)={sum(dur[k])/len(dur[k])*1e6:.1f} us")
    for c in sorted(m):
        print(f"   {c:24s} {m[c]:16.1f}")
    if "SQ_WAVES" in m and "SQ_INSTS_VALU" in m:
        w = m["SQ_WAVES"]
        print(f"   per wave: VALU {m['SQ_INSTS_VALU']/w:.0f}  LDS {m.get('SQ_INSTS_LDS',0)/w:.0f}  SALU {m.get('SQ_INSTS_SALU',0)/w:.0f}")
    if "FETCH_SIZE" in m:
        print(f"   FETCH_SIZE x2 (gfx950 correction) = {m['FETCH_SIZE']*2*1024/1e6:.1f} MB")
    if "WRITE_SIZE" in m:
        print(f"   WRITE_SIZE = {m['WRITE_SIZE']*1024/1e6:.1f} MB")
