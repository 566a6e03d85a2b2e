#!/usr/bin/env python3
"""Per-basic-block instruction mix of one kernel in the hipcc ISA listing (make -C <pkg> asm).
usage: python tools/asm_blocks.py c-filestorage-server-and-client_amd/build/rle_kernels.s decode_kernel [--min 20]
Prints each block: label, #VALU (v_*), #DPP, #SALU, #LDS (ds_*), #VMEM, #waitcnt, branch targets."""
import re
import sys


def main():
    path, kern = sys.argv[1], sys.argv[2]
    mn = int(sys.argv[sys.argv.index("--min") + 1]) if "--min" in sys.argv else 0
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(rf"^_ZN3rle\d+{kern}E.*:", l))
    blocks, cur = [], None
    for l in lines[start + 1:]:
        if l.startswith("\t.section") or re.match(r"^\.Lfunc_end", l):
            break
        m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):", l)
        if m:
            cur = {"name": m.group(1), "v": 0, "dpp": 0, "s": 0, "ds": 0, "vm": 0, "wait": 0, "br": [], "n": 0}
            blocks.append(cur)
            continue
        t = l.strip()
        if not t or t.startswith(";") or t.startswith(".") or cur is None:
            continue
        op = t.split()[0]
        cur["n"] += 1
        if op.startswith("v_"):
            cur["v"] += 1
            if "row_" in t or "wave_" in t or "quad_perm" in t:
                cur["dpp"] += 1
        elif op.startswith("ds_"):
            cur["ds"] += 1
        elif op.startswith(("buffer_", "global_", "flat_")):
            cur["vm"] += 1
        elif op == "s_waitcnt":
            cur["wait"] += 1
        elif op.startswith("s_"):
            cur["s"] += 1
            if op.startswith("s_cbranch") or op == "s_branch":
                cur["br"].append(t.split()[1])
    tot = {k: 0 for k in ("v", "dpp", "s", "ds", "vm", "wait")}
    print(f"{'block':14s} {'VALU':>5s} {'DPP':>4s} {'SALU':>5s} {'LDS':>4s} {'VMEM':>4s} {'wait':>4s}  branches")
    for b in blocks:
        for k in tot:
            tot[k] += b[k]
        if b["n"] >= mn:
            print(f"{b['name']:14s} {b['v']:5d} {b['dpp']:4d} {b['s']:5d} {b['ds']:4d} {b['vm']:4d} {b['wait']:4d}  {' '.join(b['br'])}")
    print("total", tot)


if __name__ == "__main__":
    main()
