#!/usr/bin/env python3
"""Registered large calls (csrc/rle_dropin.cpp LargeCall) into result blocks of fresh, never-touched
pages: RLEdecompress mallocs U + E bytes, which past malloc's mmap threshold are new anonymous pages.
Checks each result against the oracle and reports the first differing byte, for a sweep of sizes and
extra regions, with the process's first large allocation of each size.
usage: python tools/probes/reg_fresh_pages.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "c-filestorage-server-and-client_amd"), os.path.join(ROOT, "oracle")]
import rle_mi355x as R  # noqa: E402
import rle_oracle as O  # noqa: E402

bad = 0
for k, (U, E) in enumerate([(262143, 131073), (262145, 131071), (300000, 0), (300000, 200000), (1 << 20, 0),
                            (1 << 20, 1 << 20), (2 << 20, 12345), (262143, 131073), (262145, 131071)]):
    x = O.gen(k % 5, 70000 + k, U)
    y = O.encode(x)
    st0 = R.dropin_stats()
    got = R.decompress(y, U, E)
    st1 = R.dropin_stats()
    want = x + bytes(E)
    reg = st1["calls_registered"] - st0["calls_registered"]
    if got != want:
        bad += 1
        i = next(j for j in range(len(want)) if got[j] != want[j])
        zeros = sum(1 for j in range(0, len(want), 4096) if got[j:j + 4096] == bytes(len(got[j:j + 4096])))
        print(f"MISMATCH U={U} E={E} C={len(y)} registered={reg} first={i} got={got[i:i+8].hex()} "
              f"want={want[i:i+8].hex()} zero_pages={zeros}/{(len(want) + 4095) // 4096}", flush=True)
    else:
        print(f"ok U={U} E={E} C={len(y)} registered={reg}", flush=True)
    c = R.compress(x)
    if c != y:
        bad += 1
        print(f"COMPRESS MISMATCH U={U}", flush=True)
print("bad", bad)
sys.exit(1 if bad else 0)
