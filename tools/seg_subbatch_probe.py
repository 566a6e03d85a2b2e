#!/usr/bin/env python3
"""Round 5 question: does the segmented path's second read of its input come from the Infinity
Cache (256 MiB) when a 1 GiB batch of 1 MiB buffers is issued as sub-batches?  Times, with HIP
events (median of `reps`), the segmented encode / decode of one batch issued
  full        one call over the whole batch (today's path)
  seq<S>      sub-batches of S buffers, one call each, on one stream
  two<S>      the same sub-batches alternating over two streams (sub-batch k+1's summary beside
              sub-batch k's write pass)
and checks every decode against the input.   usage: python tools/seg_subbatch_probe.py [m1_random,...]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]
import torch  # noqa: E402

import bench  # noqa: E402
import rle_mi355x as R  # noqa: E402


def main():
    wls = (sys.argv[1] if len(sys.argv) > 1 else "m1_random,m1_runs50,m1_zero").split(",")
    reps = 5
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    s0 = torch.cuda.current_stream()
    s1 = torch.cuda.Stream()
    out = {}
    for wl in wls:
        B = bench.Batch(bench.WORKLOADS[wl], 0, 1, dev)
        B.seg = True
        B.encode(s0)
        torch.cuda.synchronize()
        clen = B.clens[0]
        ref_clen = clen.clone()
        n = B.n
        coffs = B.coffs.tolist() + [B.c_cap]
        offs = B.offs.tolist() + [B.d_in.numel()]
        res = {}
        wsd = {}
        wse = {}

        def call(kind, i0, i1, stream, key):
            tot_c = coffs[i1] - coffs[i0]
            tot_u = offs[i1] - offs[i0]
            if kind == "dec":
                if key not in wsd:
                    wsd[key] = R.seg_workspace(i1 - i0, tot_c, dev)
                R.decode_batch_seg(B.d_c, B.coffs[i0:i1], clen[i0:i1], B.d_out, B.offs[i0:i1], B.lens[i0:i1], None,
                                   B.status[i0:i1], total_in_bytes=tot_c, workspace=wsd[key], stream=stream)
            else:
                if key not in wse:
                    wse[key] = R.seg_workspace(i1 - i0, tot_u, dev)
                R.encode_batch_seg(B.d_in, B.offs[i0:i1], B.lens[i0:i1], B.d_c, B.coffs[i0:i1], clen[i0:i1],
                                   B.status[i0:i1], total_in_bytes=tot_u, workspace=wse[key], stream=stream)

        def issue(kind, mode, S):
            if mode == "full":
                call(kind, 0, n, s0, ("full",))
                return
            k = 0
            for i0 in range(0, n, S):
                i1 = min(n, i0 + S)
                st = s0 if (mode == "seq" or k % 2 == 0) else s1
                call(kind, i0, i1, st, (mode, S, k % 2 if mode == "two" else 0, i1 - i0))
                k += 1

        for kind in ("dec", "enc"):
            for mode, S in (("full", 0), ("seq", 128), ("seq", 256), ("two", 64), ("two", 128), ("two", 256)):
                name = f"{mode}{S or ''}"
                B.d_out.zero_()
                issue(kind, mode, S)   # warm + check
                s0.wait_stream(s1)
                torch.cuda.synchronize()
                if kind == "dec":
                    ok = bool(torch.equal(B.d_out, B.d_in))
                else:
                    ok = bool(torch.equal(clen, ref_clen))
                ts = []
                for _ in range(reps):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s1.wait_stream(s0)
                    e0.record(s0)
                    issue(kind, mode, S)
                    s0.wait_stream(s1)
                    e1.record(s0)
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1) * 1e3)
                ts.sort()
                res[f"{kind}_{name}"] = {"median_us": round(ts[len(ts) // 2], 1), "min_us": round(ts[0], 1), "ok": ok}
                print(wl, kind, name, res[f"{kind}_{name}"], file=sys.stderr, flush=True)
        alg = B.u_bytes + int(clen.sum().item())
        res["alg_bytes"] = alg
        out[wl] = res
        del B
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
