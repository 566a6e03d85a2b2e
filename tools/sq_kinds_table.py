#!/usr/bin/env python3
"""Per-kind SQ counter table of the codec kernels from a tools/gpu_sq_kinds.sh run (one --pmc pass of
SQ_WAVES, SQ_INSTS_VALU, SQ_INSTS_LDS, SQ_WAVE_CYCLES, SQ_WAIT_INST_ANY, SQ_LDS_BANK_CONFLICT,
SQ_LDS_IDX_ACTIVE, SQ_ACTIVE_INST_VALU and GRBM_GUI_ACTIVE per workload, means over the launches;
kernel times from the same run's --kernel-trace pass).  SQ cycle counters are quad-cycles
(MI355X_MICROARCH.md, "Per-instruction cycle constants"); tiles = the 1008-byte decode tiles or the
1024 / 1008-byte encode tiles of the workload's buffers.
usage: python tools/sq_kinds_table.py gpurun_out/<tag>_sq > profiles/<tag>_sq_kinds.md"""
import collections
import csv
import glob
import os
import statistics
import sys

WL = {  # workload: (buffers, tiles per buffer for decode (1008 B over C), for encode)
    "k64_zero": (16384, 22, 64),
    "k64_random": (16384, 66, 64),
    "k64_runs50": (16384, 66, 64),
    "k64_runs90": (16384, 31, 64),
    "cfg1": (4096, 3.5, 4),   # random 5 / zero 2 decode tiles; 4 encode tiles (1024 B)
    # configs[2]'s 1 MiB end (the segmented kernels; C / 1008 decode tiles per buffer)
    "m1_zero": (1024, 347, 1024),
    "m1_random": (1024, 1044, 1024),
    "m1_runs50": (1024, 1056, 1024),
}
SIMDS = 1024
KERNELS = ("encode_kernel", "decode_kernel", "enc_seg_", "dec_seg_")   # (with --seg: the segmented passes)


def kname(k):
    return k.split("(")[0].replace("void ", "").replace("rle::", "")


def main():
    d = sys.argv[1]
    print(f"# SQ counters per data kind ({os.path.basename(d.rstrip('/'))}; tools/gpu_sq_kinds.sh, rocprofv3)\n")
    print("One `--pmc` pass of 8 SQ counters + GRBM_GUI_ACTIVE per workload (tools/prof_driver.py, means per "
          "launch); kernel µs = median of the same workload's --kernel-trace pass. Cycle counters are quad-cycles; "
          "`VALU busy` = SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x kernel cycles), `clock` = GRBM_GUI_ACTIVE / 8 / "
          "profiled duration. `conflict share` = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE.\n")
    print("| workload | kernel | µs | clock GHz | waves | VALU/wave | VALU/tile | LDS/tile | VALU busy | "
          "WAIT_INST_ANY / WAVE_CYCLES | LDS active/CU | conflict share |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|")
    # GRBM_GUI_ACTIVE / duration reads high on dispatches shorter than ~0.3 ms (MI355X_MICROARCH.md:
    # r5's configs[1] rows came out at 3.76 GHz, above gfx950's clock).  Short dispatches take the
    # median clock of this run's long ones instead, over their --kernel-trace duration (marked *;
    # VERDICT r5 item 3).
    long_clocks = []
    for wl in WL:
        pmc = os.path.join(d, f"pmc_{wl}", "run_counter_collection.csv")
        if not os.path.exists(pmc):
            continue
        g, dur = collections.defaultdict(float), {}
        for r in csv.DictReader(open(pmc)):
            k = kname(r["Kernel_Name"])
            if not k.startswith(KERNELS):
                continue
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                g[r["Dispatch_Id"]] += float(r["Counter_Value"])
            dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        long_clocks += [g[i] / 8 / dur[i] / 1e9 for i in g if dur.get(i, 0) >= 3e-4]
    clock_ref = statistics.median(long_clocks) if long_clocks else float("nan")
    for wl, (nb, dtiles, etiles) in WL.items():
        pmc = os.path.join(d, f"pmc_{wl}", "run_counter_collection.csv")
        kt = os.path.join(d, f"kt_{wl}", "run_kernel_trace.csv")
        if not os.path.exists(pmc) or not os.path.exists(kt):
            continue
        times = collections.defaultdict(list)
        for r in csv.DictReader(open(kt)):
            times[kname(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
        vals = collections.defaultdict(lambda: collections.defaultdict(list))
        pdur = collections.defaultdict(dict)
        for r in csv.DictReader(open(pmc)):
            k = kname(r["Kernel_Name"])
            if not k.startswith(KERNELS):
                continue
            key = (r["Dispatch_Id"])
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            pdur[k][key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        for k in sorted(vals):
            m = {c: statistics.mean(v) for c, v in vals[k].items()}
            us = statistics.median(times[k]) if times.get(k) else float("nan")
            pd = statistics.mean(pdur[k].values())
            clock = m["GRBM_GUI_ACTIVE"] / 8 / pd / 1e9 if "GRBM_GUI_ACTIVE" in m else float("nan")
            short = pd < 3e-4
            waves = m["SQ_WAVES"]
            tiles = nb * (etiles if k.startswith("encode") else dtiles)
            cyc = (us * 1e-6 * clock_ref if short else pd * clock) * 1e9
            if short:
                clock = clock_ref
            busy = m["SQ_ACTIVE_INST_VALU"] * 4 / (SIMDS * cyc) if cyc else float("nan")
            print(f"| {wl} | {k} | {us:.1f} | {clock:.2f}{'*' if short else ''} | {waves:.0f} | {m['SQ_INSTS_VALU'] / waves:.0f} | "
                  f"{m['SQ_INSTS_VALU'] / tiles:.0f} | {m['SQ_INSTS_LDS'] / tiles:.1f} | {busy:.2f} | "
                  f"{m['SQ_WAIT_INST_ANY'] / m['SQ_WAVE_CYCLES']:.2f} | "
                  f"{m['SQ_LDS_IDX_ACTIVE'] / 256 / cyc:.2f} | "
                  f"{m['SQ_LDS_BANK_CONFLICT'] / max(1.0, m['SQ_LDS_IDX_ACTIVE']):.2f} |")
    print("\nRaw means per launch:\n")
    for wl in WL:
        pmc = os.path.join(d, f"pmc_{wl}", "run_counter_collection.csv")
        if not os.path.exists(pmc):
            continue
        vals = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(pmc)):
            k = kname(r["Kernel_Name"])
            if k.startswith("encode_kernel") or k.startswith("decode_kernel"):
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k in sorted(vals):
            print(f"* {wl} {k}: " + ", ".join(f"{c} {statistics.mean(v):.4g}" for c, v in sorted(vals[k].items())))


if __name__ == "__main__":
    main()
