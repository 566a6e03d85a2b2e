#!/usr/bin/env python3
"""Same-process A/B of codec builds: the product library and every build/variants/librle_*.so are
loaded side by side (separate ctypes handles), one batch per workload is built once, and encode /
decode launches of each build are timed alternately (HIP events around `reps` back-to-back
launches, `rounds` interleaved rounds; median and min per build).  Every build's round trip is
checked.   usage: python tools/ab_events.py [--workloads cfg1,dec64k] [--reps 20] [--rounds 7]"""
import argparse
import ctypes
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]
import torch  # noqa: E402

import bench  # noqa: E402

PKG = os.path.join(REPO, "c-filestorage-server-and-client_amd")


def load(path):
    L = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    vp, u32, u64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
    L.rle_encode_batch_device_sized.argtypes = [vp] * 7 + [u32, u64, vp]
    L.rle_decode_batch_device_sized.argtypes = [vp] * 8 + [u32, u64, u64, vp]
    sz = ctypes.c_size_t
    L.rle_encode_batch_device_seg.argtypes = [vp] * 7 + [u32, u64, vp, sz, vp]
    L.rle_decode_batch_device_seg.argtypes = [vp] * 8 + [u32, u64, vp, sz, vp]
    L.rle_seg_workspace_bytes.argtypes = [u32, u64]
    L.rle_seg_workspace_bytes.restype = sz
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="cfg1,dec64k")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--seg", action="store_true", help="the segmented entry points (several waves per buffer)")
    a = ap.parse_args()
    libs = {"product": load(os.path.join(PKG, "librle_mi355x.so"))}
    for p in sorted(glob.glob(os.path.join(PKG, "build", "variants", "librle_*.so"))):
        libs[os.path.basename(p)[7:-3]] = load(p)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    s = torch.cuda.current_stream()
    sp = ctypes.c_void_p(s.cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    out = {}
    for wl in a.workloads.split(","):
        B = bench.Batch(bench.WORKLOADS[wl], 0, 1, dev)
        B.encode(s)
        B.calibrate()
        ref_clen = B.clens[0].clone()
        clen = B.clens[0]

        # each build sizes its own segmented workspace (builds may cut segments differently)
        wse, wsd = {}, {}
        for k, L in libs.items():
            wse[k] = torch.empty(int(L.rle_seg_workspace_bytes(B.n, B.u_bytes)) + 256, dtype=torch.uint8, device=dev)
            wsd[k] = torch.empty(int(L.rle_seg_workspace_bytes(B.n, B.c_cap)) + 256, dtype=torch.uint8, device=dev)
        al = lambda w: ctypes.c_void_p((w.data_ptr() + 255) & ~255)
        wn = lambda w: w.numel() - 256
        name = {id(L): k for k, L in libs.items()}
        inmask = torch.zeros(B.d_in.numel(), dtype=torch.bool, device=dev)
        for o, u in zip(B.offs.tolist(), B.lens.tolist()):
            inmask[o:o + u] = True

        def enc(L):
            if a.seg:
                L.rle_encode_batch_device_seg(P(B.d_in), P(B.offs), P(B.lens), P(B.d_c), P(B.coffs), P(clen),
                                              P(B.status), B.n, B.u_bytes, al(wse[name[id(L)]]), wn(wse[name[id(L)]]), sp)
            else:
                L.rle_encode_batch_device_sized(P(B.d_in), P(B.offs), P(B.lens), P(B.d_c), P(B.coffs), P(clen),
                                                P(B.status), B.n, B.max_u, sp)

        def dec(L):
            if a.seg:
                L.rle_decode_batch_device_seg(P(B.d_c), P(B.coffs), P(clen), P(B.d_out), P(B.offs), P(B.lens), None,
                                              P(B.status), B.n, B.c_cap, al(wsd[name[id(L)]]), wn(wsd[name[id(L)]]), sp)
            else:
                L.rle_decode_batch_device_sized(P(B.d_c), P(B.coffs), P(clen), P(B.d_out), P(B.offs), P(B.lens), None,
                                                P(B.status), B.n, B.max_c, B.max_u, sp)

        res = {k: {"enc": [], "dec": [], "ok": True} for k in libs}
        for k, L in libs.items():   # correctness of every build on this batch (outputs poisoned first)
            B.d_out.copy_(B.d_in)
            B.d_out[inmask] ^= 0xFF   # every decoded byte differs from the input until written
            B.d_c.fill_(0xA5)
            enc(L)
            dec(L)
            torch.cuda.synchronize()
            res[k]["ok"] = bool(torch.equal(B.d_out, B.d_in)) and bool(torch.equal(clen, ref_clen))
        for _ in range(a.rounds):
            for k, L in libs.items():
                for kind, fn in (("enc", enc), ("dec", dec)):
                    fn(L)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    for _ in range(a.reps):
                        fn(L)
                    e1.record(s)
                    torch.cuda.synchronize()
                    res[k][kind].append(e0.elapsed_time(e1) / a.reps * 1e3)
                    print(f"  {wl} {k} {kind} {res[k][kind][-1]:.1f} us", file=sys.stderr, flush=True)
        for k in res:
            for kind in ("enc", "dec"):
                v = sorted(res[k][kind])
                res[k][kind] = {"median_us": round(v[len(v) // 2], 2), "min_us": round(v[0], 2)}
        out[wl] = res
        print(wl, json.dumps(res), flush=True)
        del B
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
