#!/usr/bin/env python3
"""configs[2] HBM-roofline sweep: device-resident encode / decode of synthetic batches of one buffer
size (4 KiB .. 1 MiB) and one run density (zero-fill / random / 50 % runs), about 1 GiB of input per
point, each through the one-wave-per-buffer kernels and the segmented (several waves per buffer)
forms.  Per point: kernel time from HIP events on the launch stream, achieved GB/s = algorithmic
bytes (U + C) / time, and the fraction of the 8 TB/s HBM peak; every round trip is checked equal.

usage: python tools/roofline_sweep.py [--reps 5] > profiles/<tag>_sweep.json"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]
import torch  # noqa: E402

import bench  # noqa: E402

PEAK = 8000.0   # GB/s, MI355X HBM3E
KINDS = {"zero": 0, "random": 1, "runs50": 2}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--bytes", type=int, default=1 << 30, help="input bytes per point")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    s = torch.cuda.current_stream()
    rows = []
    for size in (4096, 16384, 65536, 262144, 1 << 20):
        n = max(256, a.bytes // size)
        for kname, kind in KINDS.items():
            wl = dict(n=n, size=size, kinds=(kind,), ref_kinds=str(kind), desc="")
            B = bench.Batch(wl, 0, 1, dev)
            for seg in (False, True):
                B.seg = seg
                B.encode(s)
                B.decode(s)
                torch.cuda.synchronize()
                ok = bool(torch.equal(B.d_out, B.d_in)) and int(B.status.abs().sum().item()) == 0
                te = bench.time_kernels(lambda: B.encode(s), a.reps, s)
                td = bench.time_kernels(lambda: B.decode(s), a.reps, s)
                C = int(B.clen.sum().item())
                alg = B.u_bytes + C
                rows.append({"size": size, "kind": kname, "buffers": n, "path": "seg" if seg else "wave",
                             "U": B.u_bytes, "C": C, "ok": ok,
                             "encode_us": te * 1e6, "decode_us": td * 1e6,
                             "encode_GBps": alg / te / 1e9, "decode_GBps": alg / td / 1e9,
                             "encode_frac": alg / te / 1e9 / PEAK, "decode_frac": alg / td / 1e9 / PEAK})
                print(f"{size:8d} {kname:7s} {rows[-1]['path']:4s} ok={ok} enc {rows[-1]['encode_GBps']:7.0f} "
                      f"dec {rows[-1]['decode_GBps']:7.0f} GB/s", file=sys.stderr, flush=True)
            del B
            torch.cuda.empty_cache()
    print(json.dumps({"peak_GBps": PEAK, "bytes_per_point": a.bytes, "rows": rows}))
    return 0 if all(r["ok"] for r in rows) else 1


if __name__ == "__main__":
    sys.exit(main())
