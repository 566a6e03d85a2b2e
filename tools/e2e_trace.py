#!/usr/bin/env python3
"""Per-call trace of the drop-in behind the UNCHANGED reference server (RLE_MI355X_TRACE, csrc/
rle_dropin.cpp): batteries 1 and 2 of tests/test_e2e_server.py on a started server (SETTLE seconds
after its socket appears) and battery 3 of tools/e2e_compare.py, each on a fresh server_gpu.  For
each battery prints one JSON object: the battery's wall time, the codec calls (count and total ms
per entry point), the time the calls spent getting their thread context, and the slowest calls
with their sizes -- where the server's time over server_ref goes.
usage: python tools/e2e_trace.py"""
import collections
import json
import os
import shutil
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "tools")]
import e2e_compare as EC  # noqa: E402
import test_e2e_server as E  # noqa: E402

OPS = {"c": "RLEcompress", "d": "RLEdecompress", "a": "RLEappend", "n": "RLEdecompressN",
       "I": "start-up: runtime", "P": "start-up: context", "N": "start-up: new context"}


def summarize(path):
    recs = []
    for line in open(path):
        op, tid, a, b, c, t0, dt, cn = line.split()
        recs.append(dict(op=OPS[op], tid=int(tid), a=int(a), b=int(b), c=int(c), t0=int(t0), dt=int(dt),
                         ctx=int(cn)))
    by = collections.defaultdict(lambda: [0, 0])
    for r in recs:
        by[r["op"]][0] += 1
        by[r["op"]][1] += r["dt"]
    start = [r for r in recs if r["op"].startswith("start-up")]
    recs = [r for r in recs if not r["op"].startswith("start-up")]
    slow = sorted(recs, key=lambda r: -r["dt"])[:12]
    return {"calls": {k: {"n": v[0], "ms": round(v[1] / 1e6, 3)} for k, v in by.items()},
            "ctx_ms": round(sum(r["ctx"] for r in recs) / 1e6, 3),
            "threads": len({r["tid"] for r in recs}),
            "start_up_ms": [(r["op"][10:], r["a"], r["b"], round(r["dt"] / 1e6, 2)) for r in sorted(start, key=lambda r: r["t0"])],
            "slowest": [{"op": r["op"], "sizes": [r["a"], r["b"], r["c"]], "us": round(r["dt"] / 1e3, 1),
                         "ctx_us": round(r["ctx"] / 1e3, 1)} for r in slow]}


def main():
    exe = os.path.join(E.BIN, "server_gpu")
    for variant, extra in (("default", {}), ("zcseg0", {"RLE_MI355X_ZC_SEG": "0"})):
        for name in ("battery1", "battery2", "battery3"):
            run(exe, variant, extra, name)


def run(exe, variant, extra, name):
    with tempfile.TemporaryDirectory() as tmp:
        tr = os.path.join(tmp, "trace.txt")
        env = dict(extra, RLE_MI355X_TRACE=tr)
        if name == "battery1":
            r = E.battery1(exe, os.path.join(tmp, "b"), env, EC.SETTLE)
            E._check_battery1(r)
            wall = r[3]
        elif name == "battery2":
            r = E.battery2(exe, os.path.join(tmp, "b"), env, EC.SETTLE)
            E._check_battery2(r)
            wall = r[3]
        else:
            cold, hot = EC.battery3(exe, os.path.join(tmp, "b"), env)
            wall = [cold, hot]
        out = {"variant": variant, "battery": name, "wall_s": wall}
        out.update(summarize(tr) if os.path.exists(tr) else {"trace": "missing"})
        keep = os.environ.get("E2E_TRACE_KEEP")   # a directory for the raw per-call traces
        if keep and os.path.exists(tr):
            os.makedirs(keep, exist_ok=True)
            shutil.copyfile(tr, os.path.join(keep, f"{variant}_{name}.txt"))
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
