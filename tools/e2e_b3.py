#!/usr/bin/env python3
"""Battery 3 of tools/e2e_compare.py alone (8 concurrent clients, 64 small files each, warm server),
more repetitions, over server_ref and server_gpu with environment variants of the drop-in's wait:
the default (poll the status word, spin RLE_MI355X_SPIN_NS = 50 us, then yield), yielding from the
start (SPIN_NS=0), and hipStreamSynchronize instead of polling (POLL=0).  The runs interleave the
servers, so a box's drift spreads over all of them.  Prints one JSON object.
usage: python tools/e2e_b3.py [--reps 5]"""
import argparse
import json
import os
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "tools")]
import e2e_compare as C  # noqa: E402
import test_e2e_server as E  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only", default="", help="comma-separated variant names (default: all)")
    a = ap.parse_args()
    variants = (("server_ref", "server_ref", None), ("server_gpu", "server_gpu", None),
                ("server_gpu_spin0", "server_gpu", {"RLE_MI355X_SPIN_NS": "0"}),
                ("server_gpu_poll0", "server_gpu", {"RLE_MI355X_POLL": "0"}))
    if a.only:
        variants = tuple(v for v in variants if v[0] in a.only.split(","))
    res = {name: {"battery3_cold_s": [], "battery3_warm_s": []} for name, _, _ in variants}
    for r in range(a.reps):
        for name, exe, env in variants:
            with tempfile.TemporaryDirectory() as tmp:
                cold, hot = C.battery3(os.path.join(E.BIN, exe), tmp, env)
            res[name]["battery3_cold_s"].append(round(cold, 4))
            res[name]["battery3_warm_s"].append(round(hot, 4))
        print("rep", r, "done", file=sys.stderr, flush=True)
    for v in res.values():
        w = sorted(v["battery3_warm_s"])
        v["warm_median_s"] = w[len(w) // 2]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
