#!/usr/bin/env python3
"""Turn one GPU round's raw rocprofv3 output (tools/gpu_round.sh) into the committed profiles/:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary of `bench.py --steps 20`
  profiles/<tag>_kernel_split.md    the same trace split per (kernel, grid): bench runs the cfg1 batch
                                    and then the dec64k north-star batch, which the stats file mixes
  profiles/<tag>_pmc.md             FETCH_SIZE / WRITE_SIZE per codec launch for each workload
  profiles/pmc_traffic.json         {workload: {kernel: HBM bytes per launch}} read by bench.py

HBM bytes = 2 x FETCH_SIZE x 1024 + WRITE_SIZE x 1024 (FETCH_SIZE and WRITE_SIZE are in KiB;
gfx950 tallies wide coalesced reads at half their bytes: /opt/skills/guides/MI355X_MICROARCH.md,
"HBM [CDNA4]").  Each counter comes from its own --pmc pass.
usage: python tools/make_profiles.py gpurun_out/r1a r1
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(REPO, "profiles")


def short(name):
    # template arguments dropped: decode_kernel<96u> / <192u> (the staging size) are one kernel
    return name.split("(")[0].split("<")[0].replace("rle::", "").replace("void ", "")


def kernel_split(src):
    rows = defaultdict(list)
    for r in csv.DictReader(open(os.path.join(src, "prof", "run_kernel_trace.csv"))):
        if "rle::" not in r["Kernel_Name"]:
            continue
        g = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
        rows[(short(r["Kernel_Name"]), g, int(r["LDS_Block_Size"]), int(r["VGPR_Count"]))].append(
            int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = ["| kernel | workgroups | LDS B | VGPR | launches | avg us | min us | max us |",
           "|---|---|---|---|---|---|---|---|"]
    res = {}
    for (k, g, lds, v), d in sorted(rows.items()):
        avg = sum(d) / len(d) / 1e3
        out.append(f"| {k} | {g} | {lds} | {v} | {len(d)} | {avg:.2f} | {min(d)/1e3:.2f} | {max(d)/1e3:.2f} |")
        res[(k, g)] = avg
    return "\n".join(out), res


def pmc(src, workload):
    per = defaultdict(dict)
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = os.path.join(src, f"pmc_{workload}_{c}", "run_counter_collection.csv")
        if not os.path.exists(f):
            return None
        acc = defaultdict(list)
        for r in csv.DictReader(open(f)):
            if "rle::" in r["Kernel_Name"] and r["Counter_Name"] == c:
                acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
        for k, v in acc.items():
            # the first encode launch of prof_driver is a warm-up identical to the rest
            per[k][c] = sum(v) / len(v)
            per[k][c + "_n"] = len(v)
    return per


def main():
    src, tag = sys.argv[1], sys.argv[2]
    os.makedirs(PROF, exist_ok=True)
    shutil.copyfile(os.path.join(src, "prof", "run_kernel_stats.csv"),
                    os.path.join(PROF, f"{tag}_kernel_stats.csv"))
    table, _ = kernel_split(src)
    with open(os.path.join(PROF, f"{tag}_kernel_split.md"), "w") as f:
        f.write(f"# {tag}: rocprofv3 --kernel-trace of `python3 bench.py --steps 20 --no-cpu`\n\n"
                "Split per (kernel, grid). The smaller grids are the configs[1] batch (4096 x 4 KiB),\n"
                "the larger ones the dec64k north-star batch (16384 x 64 KiB); bench.py times both.\n\n")
        f.write(table + "\n")
    traffic = {}
    lines = [f"# {tag}: HBM traffic per codec launch (rocprofv3 --pmc, one counter per pass)\n",
             "HBM bytes = 2 x FETCH_SIZE x 1 KiB + WRITE_SIZE x 1 KiB (gfx950 FETCH_SIZE halving).\n",
             "| workload | kernel | launches | FETCH_SIZE KiB | WRITE_SIZE KiB | read MB (x2) | write MB | HBM MB |",
             "|---|---|---|---|---|---|---|---|"]
    for wl in ("cfg1", "dec64k"):
        p = pmc(src, wl)
        if not p:
            continue
        traffic[wl] = {}
        for k in sorted(p):
            m = p[k]
            rd = 2 * m["FETCH_SIZE"] * 1024
            wr = m["WRITE_SIZE"] * 1024
            traffic[wl][k.replace("_kernel", "")] = int(rd + wr)
            lines.append(f"| {wl} | {k} | {m['FETCH_SIZE_n']} | {m['FETCH_SIZE']:.0f} | {m['WRITE_SIZE']:.0f} | "
                         f"{rd/1e6:.1f} | {wr/1e6:.1f} | {(rd+wr)/1e6:.1f} |")
    with open(os.path.join(PROF, f"{tag}_pmc.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    hp = os.path.join(src, "host.txt")
    host = open(hp).read().split()[0] if os.path.exists(hp) else "unrecorded"
    traffic["_source"] = (f"profiles/{tag}_pmc.md (rocprofv3 --pmc FETCH_SIZE, WRITE_SIZE; bytes per launch; "
                          f"GPU round {tag}, box {host}; a different process from the bench line's)")
    with open(os.path.join(PROF, "pmc_traffic.json"), "w") as f:
        json.dump(traffic, f, indent=1)
    print(table)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
