#!/usr/bin/env python3
"""Registered large decompress calls (csrc/rle_dropin.cpp decompress_registered) repeated with the
same result-block size, so that malloc hands out mmap'd blocks at recurring addresses: every
result checked against the oracle, mismatches reported with their first differing byte and the
share of all-zero pages.  Interleaves zero-copy small calls, as tests/test_gpu_hostpath.py's
polled-calls test does.   usage: python tools/probes/reg_stress.py [iterations]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "c-filestorage-server-and-client_amd"), os.path.join(ROOT, "oracle")]
import rle_mi355x as R  # noqa: E402
import rle_oracle as O  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 200
sizes = [65537, 80641, 131072, 262143, 262145, 300000]
cases = []
for k, U in enumerate(sizes):
    x = O.gen(k % 5, 70000 + k, U)
    cases.append((x, O.encode(x), U))
small = [(O.gen(k % 5, k, 3000 + 100 * k), None) for k in range(8)]
small = [(x, O.encode(x)) for x, _ in small]
bad = 0
for it in range(iters):
    x, y, U = cases[it % len(cases)]
    E = 393216 - U if U < 393216 else 0
    got = R.decompress(y, U, E)
    want = x + bytes(E)
    if got != want:
        bad += 1
        i = next(j for j in range(len(want)) if got[j] != want[j])
        zp = sum(1 for j in range(0, len(want), 4096) if got[j:j + 4096] == bytes(len(got[j:j + 4096])))
        print(f"MISMATCH it={it} U={U} E={E} first={i} got={got[i:i + 8].hex()} want={want[i:i + 8].hex()} "
              f"zero_pages={zp}/{(len(want) + 4095) // 4096}", flush=True)
    sx, sy = small[it % len(small)]
    if R.decompress(sy, len(sx)) != sx or R.compress(sx) != sy:
        bad += 1
        print(f"SMALL MISMATCH it={it}", flush=True)
st = R.dropin_stats()
print("bad", bad, "of", iters, "registered", st["calls_registered"], "fallback", st["calls_reg_fallback"], flush=True)
sys.exit(1 if bad else 0)
