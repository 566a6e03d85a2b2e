#!/usr/bin/env python3
"""Round 5 question: does the one-pass encode (csrc/rle_coop.hip enc_stream_body: a workgroup per
buffer walking it in rounds, each input byte read once) beat the five-launch segmented encode
(summary pass + write pass: the input read twice) on large buffers?  Times, with HIP events
(median of `reps`), the segmented encode, the one-wave encode and the one-pass encode at 16 and 8
waves of each workload, and checks every output against the segmented one.
usage: python tools/stream_probe.py [m1_random,m1_runs50,...]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]
import torch  # noqa: E402

import bench  # noqa: E402
import rle_mi355x as R  # noqa: E402


def timed(fn, s, reps=7):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        fn()
        e1.record(s)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    wls = (sys.argv[1] if len(sys.argv) > 1 else "m1_zero,m1_random,m1_runs50,mixed,one4m,k64_random,k64_runs50").split(",")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    s = torch.cuda.current_stream()
    out = {}
    for wl in wls:
        B = bench.Batch(bench.WORKLOADS[wl], 0, 1, dev)
        B.seg = True
        B.d_c.fill_(0xA5)
        B.encode(s)
        torch.cuda.synchronize()
        ref_len = B.clens[0].clone()
        ref = B.d_c.clone()
        alg = B.u_bytes + int(ref_len.sum().item())
        res = {"alg_bytes": alg}
        clen = B.clens[0]

        def seg():
            B.seg = True
            B.encode(s)

        def wave():
            B.seg = False
            B.encode(s)

        def one_pass():
            R.encode_batch_stream(B.d_in, B.offs, B.lens, B.d_c, B.coffs, clen, B.status, stream=s)

        for name, fn, w in (("seg", seg, None), ("wave", wave, None), ("pass16", one_pass, 16), ("pass8", one_pass, 8), ("pass4", one_pass, 4)):
            if w:
                R.set_stream_waves(w)
            B.d_c.fill_(0xA5)
            fn()
            torch.cuda.synchronize()
            ok = bool(torch.equal(clen, ref_len)) and bool(torch.equal(B.d_c, ref))
            us = timed(fn, s)
            res[name] = {"us": round(us, 1), "frac": round(alg / (us * 1e-6) / 8e12, 4), "ok": ok}
            print(wl, name, res[name], file=sys.stderr, flush=True)
        R.set_stream_waves(16)
        out[wl] = res
        del B
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
