#!/usr/bin/env python3
"""Per-wave timelines of one encode and one decode launch (RLE_TIMELINE=1 builds: make variant
NAME=tl DEFS=-DRLE_TIMELINE=1; selected with RLE_MI355X_LIB).  Prints, in microseconds relative to
the first wave's entry: the spread of wave entries, walk starts, the start of each tile, the ends,
and per tile index the median interval between consecutive tile starts.
usage: RLE_MI355X_LIB=.../librle_tl.so python tools/timeline.py [--workload cfg1] [--n 256]"""
import argparse
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]
import torch  # noqa: E402

import bench  # noqa: E402
import rle_mi355x as R  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="cfg1")
ap.add_argument("--n", type=int, default=0, help="buffers (default: the workload's); e.g. 256 for lone waves")
a = ap.parse_args()
L = R.lib()
L.rle_mi355x_timeline.restype = ctypes.c_int
L.rle_mi355x_timeline.argtypes = [ctypes.c_void_p, ctypes.c_int]
NW, NE = 16384, 16
buf = np.zeros(NW * NE, np.uint64)


def grab():
    torch.cuda.synchronize()
    assert L.rle_mi355x_timeline(buf.ctypes.data, 1) == 0, "not a timeline build"
    return buf.reshape(NW, NE).astype(np.int64).copy()


def pct(x):
    return " ".join(f"{v:7.2f}" for v in np.percentile(x, [0, 10, 50, 90, 100]))


def report(name, tl, n):
    tl = tl[:n]
    ok = tl[:, 0] > 0
    tl = tl[ok]
    t0 = tl[:, 13].min()
    us = lambda c: (c - t0) / 100.0   # s_memrealtime: 100 MHz
    print(f"== {name}: {len(tl)} waves  (percentiles 0/10/50/90/100, us from the first wave's first instruction)")
    print(f"  first inst {pct(us(tl[:, 13]))}")
    print(f"  entry      {pct(us(tl[:, 0]))}")
    print(f"  first->entry {pct((tl[:, 0] - tl[:, 13]) / 100.0)}")
    print(f"  walk start {pct(us(tl[:, 1]))}")
    for t in range(8):
        c = tl[:, 2 + t]
        m = c > 0
        if m.sum() == 0:
            break
        print(f"  tile {t} start {pct(us(c[m]))}   n={m.sum()}")
    print(f"  end        {pct(us(tl[:, 10]))}")
    # per-wave intervals
    for t in range(7):
        a_, b_ = tl[:, 2 + t], tl[:, 3 + t]
        m = (a_ > 0) & (b_ > 0)
        if m.sum() == 0:
            break
        print(f"  tile {t}->{t + 1} interval {pct((b_[m] - a_[m]) / 100.0)}")
    last = np.where(tl[:, 2:10] > 0, tl[:, 2:10], 0).max(axis=1)
    print(f"  last tile -> end {pct((tl[:, 10] - last) / 100.0)}")
    print(f"  entry -> tile0 {pct((tl[:, 2] - tl[:, 0]) / 100.0)}")
    if (tl[:, 14] > 0).any():   # decode: metadata arrival and first loads issued
        m = (tl[:, 14] > 0) & (tl[:, 15] > 0)
        print(f"  entry -> metadata {pct((tl[m, 14] - tl[m, 0]) / 100.0)}")
        print(f"  metadata -> loads issued {pct((tl[m, 15] - tl[m, 14]) / 100.0)}")
        print(f"  loads issued -> walk start {pct((tl[m, 1] - tl[m, 15]) / 100.0)}")
        print(f"  walk start -> tile0 {pct((tl[m, 2] - tl[m, 1]) / 100.0)}")
    xcc = tl[:, 12] & 0xF
    hw = tl[:, 11]
    # per SIMD (XCC, SE, SH, CU, SIMD from HW_ID): tiles walked by its waves, and its last end
    simd = (xcc << 20) | (hw & 0xFF30)   # SIMD_ID 5:4, CU_ID 11:8, SH_ID 12, SE_ID 15:13
    ntile = (tl[:, 2:10] > 0).sum(axis=1)
    keys, inv = np.unique(simd, return_inverse=True)
    tsum = np.bincount(inv, weights=ntile)
    wcnt = np.bincount(inv)
    lend = np.zeros(len(keys))
    np.maximum.at(lend, inv, us(tl[:, 10]))
    print(f"  SIMDs {len(keys)}  waves/SIMD {pct(wcnt)}  tiles/SIMD {pct(tsum)}")
    for lo, hi in ((0, 10), (10, 16), (16, 100)):
        m = (tsum >= lo) & (tsum < hi)
        if m.any():
            print(f"    SIMDs with {lo}-{hi} tiles: {m.sum():4d}, last end {pct(lend[m])}")
    print(f"  XCCs {np.bincount(xcc, minlength=8).tolist()}  wave-slots {np.bincount(hw & 0xF, minlength=8).tolist()}")


torch.cuda.set_device(0)
wl = dict(bench.WORKLOADS[a.workload])
if a.n:
    wl["n"] = a.n
B = bench.Batch(wl, 0, 1, torch.device("cuda", 0))
s = torch.cuda.current_stream()
B.encode(s)
B.calibrate()
for _ in range(3):
    B.encode(s)
    B.decode(s)
grab()
B.encode(s)
enc = grab()
B.decode(s)
dec = grab()
# the same launches right behind another launch of the same kernel (as in the bench loop): the
# second overwrites the first's marks
B.encode(s)
B.encode(s)
enc2 = grab()
B.decode(s)
B.decode(s)
dec2 = grab()
report("encode " + a.workload, enc, B.n)
report("decode " + a.workload, dec, B.n)
report("encode behind encode " + a.workload, enc2, B.n)
report("decode behind decode " + a.workload, dec2, B.n)
ok = torch.equal(B.d_out, B.d_in)
print("roundtrip", "ok" if ok else "MISMATCH")
