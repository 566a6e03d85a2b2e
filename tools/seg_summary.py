#!/usr/bin/env python3
"""Sum the codec kernel time per launch for one-wave vs segmented modes (tools/seg_compare.sh).
usage: python tools/seg_summary.py gpurun_out/segcmp1"""
import csv
import glob
import os
import sys
from collections import defaultdict

ENC = ("encode_kernel", "seg_plan_kernel:enc", "enc_seg_summary_kernel", "enc_seg_scan_kernel", "enc_seg_write_kernel")
root = sys.argv[1]
for d in sorted(glob.glob(os.path.join(root, "*_*"))):
    if not os.path.isdir(d):
        continue
    mode, wl = os.path.basename(d).split("_", 1)
    rows = []
    for f in glob.glob(os.path.join(d, "*kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("rle::", "").replace("void ", "")
            if k.startswith("gen_") or "rle" not in r["Kernel_Name"]:
                continue
            rows.append((int(r["Start_Timestamp"]), k, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    rows.sort()
    # group consecutive kernels into launches: encode = (plan, enc_*) or encode_kernel; decode likewise
    per = defaultdict(list)
    cur, acc = None, 0.0
    for _, k, us in rows:
        kind = "enc" if k.startswith("enc") or k == "encode_kernel" else ("dec" if k.startswith("dec") or k == "decode_kernel" else None)
        if k == "seg_plan_kernel":
            if cur:
                per[cur].append(acc)
            cur, acc = "pending", us
            continue
        if kind is None:
            continue
        if cur == "pending":
            cur = kind
            acc += us
        elif k in ("encode_kernel", "decode_kernel"):
            if cur:
                per[cur].append(acc)
            cur, acc = kind, us
        else:
            acc += us
    if cur:
        per[cur].append(acc)
    out = []
    for kind in ("enc", "dec"):
        v = per.get(kind, [])[1:] or per.get(kind, [])
        if v:
            out.append(f"{kind} {sum(v)/len(v):9.1f} us (n={len(v)})")
    log = open(d + ".log").read().strip().splitlines()
    ok = [l for l in log if l.startswith("ok") or l.startswith("MISMATCH")]
    print(f"{wl:8s} {mode:4s} " + " | ".join(out) + "   " + (ok[-1] if ok else "?"))
