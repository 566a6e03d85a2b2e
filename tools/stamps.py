#!/usr/bin/env python3
"""Decode segment shares from a diagnostic (RLE_STAMPS=1) build.
usage: RLE_MI355X_LIB=.../build/variants/librle_stamps.so python tools/stamps.py k64_random [k64_zero ...]"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]
import torch  # noqa: E402

import bench  # noqa: E402

R = bench.R
L = R.lib()
L.rle_mi355x_stamps.restype = ctypes.c_int
L.rle_mi355x_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
SEG = ["wait+loop", "scan/lengths", "scatter", "fl:reads", "fl:fill+scan", "fl:store", "fl:zero+sync",
       "move/drain/finish"]
SEG_ENC = ["wait+loop", "bounds/scans", "pass1", "pass2+sync", "flush", "move/state", "drain", "finish"]
torch.cuda.set_device(0)
for arg in sys.argv[1:]:
    enc = arg.startswith("enc:")
    wl = arg[4:] if enc else arg
    B = bench.Batch(bench.WORKLOADS[wl], 0, 1, torch.device("cuda", 0))
    s = torch.cuda.current_stream()
    B.encode(s)
    B.decode(s)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 9)()
    assert L.rle_mi355x_stamps(buf, 1) == 0, "not a stamps build"
    reps = 3
    for _ in range(reps):
        if enc:
            B.encode(s)
        else:
            B.decode(s)
    torch.cuda.synchronize()
    L.rle_mi355x_stamps(buf, 1)
    ok = torch.equal(B.d_out, B.d_in)
    v = list(buf)
    tot, waves = sum(v[:8]), v[8]
    tiles = sum((int(c) + 1007) // 1008 for c in (B.lens if enc else B.clen).tolist()) * reps
    print(f"== {'encode' if enc else 'decode'} {wl}: ok={ok} waves={waves} tiles={tiles} cycles/wave={tot / max(waves, 1):.0f} "
          f"cycles/tile={tot / max(tiles, 1):.0f}")
    for k, name in enumerate(SEG_ENC if enc else SEG):
        print(f"   {name:14s} {100 * v[k] / max(tot, 1):6.1f} %   {v[k] / max(tiles, 1):8.0f} cyc/tile")
    del B
    torch.cuda.empty_cache()
