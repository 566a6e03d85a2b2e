#!/usr/bin/env python3
"""Per-(kernel, grid) duration summary of rocprofv3 kernel-trace dirs.
usage: python tools/kt_summary.py gpurun_out/it1/kt_dec64k [more dirs...]"""
import csv
import glob
import os
import sys
from collections import defaultdict

for d in sys.argv[1:]:
    rows = defaultdict(list)
    for f in glob.glob(os.path.join(d, "*kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            if "rle::" not in r["Kernel_Name"]:
                continue
            k = r["Kernel_Name"].split("(")[0].replace("rle::", "")
            g = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
            rows[(k, g)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print("==", d)
    for (k, g), v in sorted(rows.items()):
        v2 = v[1:] if len(v) > 2 else v
        print(f"  {k:16s} grid {g:6d}  n={len(v):3d}  avg {sum(v2)/len(v2):9.2f} us  min {min(v):9.2f}")
