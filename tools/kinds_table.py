#!/usr/bin/env python3
"""Per-kind roofline table of the 64 KiB decode / encode (the north-star batch and its four data
kinds) from a tools/gpu_kinds.sh run: rocprof median kernel time per workload, the batch's
algorithmic bytes (U + C, C from the oracle's encoding of the same seeded buffers), GB/s and the
fraction of 8 TB/s.  --skip K drops each kernel's first K launches (round 6: the warm launches of
tools/gpu_kinds.sh, so the table is steady state like bench.py's north-star timing).
   usage: python tools/kinds_table.py gpurun_out/<tag>_kinds [--skip K] > profiles/<tag>_kinds.md"""
import collections
import csv
import glob
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "oracle")]
import rle_oracle as O  # noqa: E402

N, U = 16384, 65536
KINDS = {"k64_zero": (0,), "k64_random": (1,), "k64_runs50": (2,), "k64_runs90": (3,), "dec64k": (0, 1, 2, 3)}


def c_bytes(kinds):
    return sum(len(O.encode(O.gen(kinds[i % len(kinds)], i, U))) for i in range(N))


def main():
    d = sys.argv[1]
    skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 0
    print(f"# Per-kind 64 KiB codec launches ({os.path.basename(d.rstrip('/'))}, rocprofv3 --kernel-trace, "
          f"median of each kernel's launches after its first {skip})\n")
    print("16384 x 64 KiB per launch (1 GiB of U). Algorithmic bytes = U + C; fraction of 8 TB/s. "
          "Decode excludes the issue-order sort (its own launch, listed).\n")
    print("| workload | C MB | encode µs | encode frac | decode µs | decode frac | sort µs |")
    print("|---|---|---|---|---|---|---|")
    for wl, kinds in KINDS.items():
        path = os.path.join(d, f"kt_{wl}", "run_kernel_trace.csv")
        if not os.path.exists(path):
            continue
        dur = collections.defaultdict(list)
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"]
            key = "enc" if "encode_kernel" in name else "dec" if "decode_kernel" in name else \
                "sort" if "dec_order" in name else None
            if key:
                dur[key + name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
        med = lambda v: sorted(v[skip:] if len(v) > skip else v)[len(v[skip:] if len(v) > skip else v) // 2]
        enc = [med(v) for k, v in dur.items() if k.startswith("enc")][0]
        dec = [med(v) for k, v in dur.items() if k.startswith("dec") and "decode_kernel" in k][0]
        srt = sum(med(v) for k, v in dur.items() if k.startswith("sort"))
        C = c_bytes(kinds)
        alg = N * U + C
        fr = lambda t: alg / (t * 1e-6) / 8e12
        print(f"| {wl} | {C / 1e6:.1f} | {enc:.1f} | {fr(enc):.3f} | {dec:.1f} | {fr(dec):.3f} | {srt:.1f} |")


if __name__ == "__main__":
    main()
