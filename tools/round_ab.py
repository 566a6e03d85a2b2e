#!/usr/bin/env python3
"""Large-batch decode: one wave per buffer (decode_kernel<96>) against the decode in rounds
(csrc/rle_round.h, 4 / 8 / 16 waves per buffer), same process, steady state (GPU box).

Per workload: one untimed round of every setting, then --rounds rounds in which every setting is
timed (bench.time_kernels: --reps back-to-back launches) one after the other; the median per setting,
as µs, GB/s of (U + C) and fraction of 8 TB/s, and whether the output equals the input.
  usage: python tools/round_ab.py [--workloads dec64k,k64_zero,...] [--widths 0,4,8,16] [--rounds 3]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import torch  # noqa: E402

R = bench.R


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="dec64k,k64_zero,k64_random,k64_runs50,k64_runs90")
    ap.add_argument("--widths", default="0,4,8,16")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)
    widths = [int(w) for w in a.widths.split(",")]
    prev = R.set_dec_round(-1)
    for name in a.workloads.split(","):
        B = bench.Batch(bench.WORKLOADS[name], 0, 1, dev)
        B.encode(stream)
        B.calibrate()
        alg = B.u_bytes + int(B.clen.sum().item())
        dec = lambda: B.decode(stream)
        ok, ts = {}, {w: [] for w in widths}
        for w in widths:   # untimed round; output check
            R.set_dec_round(w)
            B.d_out.fill_(0xA5)
            dec()
            torch.cuda.synchronize()
            ok[w] = bool(torch.equal(B.d_out, B.d_in)) and int(B.status.abs().sum().item()) == 0
            bench.time_kernels(dec, a.reps, stream)
        for _ in range(a.rounds):
            for w in widths:
                R.set_dec_round(w)
                ts[w].append(bench.time_kernels(dec, a.reps, stream))
        res = {"workload": name, "alg_bytes": alg}
        for w in widths:
            t = sorted(ts[w])[len(ts[w]) // 2]
            res[f"w{w}"] = {"us": round(t * 1e6, 2), "frac": round(alg / t / 1e9 / 8000, 4), "verified": ok[w],
                            "rounds_us": [round(x * 1e6, 1) for x in ts[w]]}
        print(json.dumps(res), flush=True)
        del B
        torch.cuda.empty_cache()
    R.set_dec_round(prev)


if __name__ == "__main__":
    main()
