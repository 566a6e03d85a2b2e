#!/usr/bin/env python3
"""HBM write-only and read+write rates on this box (the ceilings of the store-bound decode kinds:
zero-filled 64 KiB decode writes 1.07 GB per launch and reads 0.36 GB).  Times, with HIP events,
a 1 GiB fill (torch fill_, hipMemsetAsync) and a 1 GiB device-to-device copy, median of 10.
usage: python tools/write_rate_probe.py"""
import json

import torch


def t(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e-3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    n = 1 << 30
    a = torch.empty(n, dtype=torch.uint8, device="cuda")
    b = torch.empty(n, dtype=torch.uint8, device="cuda")
    out = {}
    s = t(lambda: a.fill_(7))
    out["fill_1GiB"] = {"s": s, "write_TBps": n / s / 1e12}
    s = t(lambda: a.zero_())
    out["zero_1GiB"] = {"s": s, "write_TBps": n / s / 1e12}
    s = t(lambda: b.copy_(a))
    out["copy_1GiB"] = {"s": s, "rw_TBps": 2 * n / s / 1e12}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
