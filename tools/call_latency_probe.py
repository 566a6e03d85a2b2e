#!/usr/bin/env python3
"""Per-call latency of the drop-in RLEcompress / RLEdecompress on one thread, over the file sizes of
the e2e battery 3 and the zero-copy range (4 KiB - 128 KiB), random and runs-like data.  The library
is the product one unless RLE_MI355X_LIB names another build; RLE_MI355X_ZC_SEG etc. apply as in the
server.  Every call's result is checked against the first.  Prints one JSON object.
usage: python tools/call_latency_probe.py [seconds_per_point]"""
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "c-filestorage-server-and-client_amd"), os.path.join(REPO, "tools")]
import rle_mi355x as R  # noqa: E402
from hostpath_bench import gen  # noqa: E402


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 0.3
    L = R.lib()
    L.RLEcompress.restype = ctypes.c_void_p
    L.RLEdecompress.restype = ctypes.c_void_p
    out = []
    for kind in ("random", "runs"):
        for U in (4096, 8192, 16384, 24576, 32768, 40000, 49152, 65536, 98304, 131072, 262144, 524288, 1048576):
            x = gen(kind, U, U + 1)
            c = ctypes.c_size_t(0)
            p = L.RLEcompress(x, U, ctypes.byref(c))
            y = ctypes.string_at(p, c.value)
            R._libc.free(ctypes.c_void_p(p))
            q = L.RLEdecompress(y, len(y), U, 0)
            ok = ctypes.string_at(q, U) == x
            R._libc.free(ctypes.c_void_p(q))
            n, t0 = 0, time.perf_counter()
            while time.perf_counter() - t0 < secs:
                p = L.RLEcompress(x, U, ctypes.byref(c))
                if n == 0:
                    ok = ok and ctypes.string_at(p, c.value) == y
                R._libc.free(ctypes.c_void_p(p))
                n += 1
            tc = (time.perf_counter() - t0) / n
            n, t0 = 0, time.perf_counter()
            while time.perf_counter() - t0 < secs:
                q = L.RLEdecompress(y, len(y), U, 0)
                if n == 0:
                    ok = ok and ctypes.string_at(q, U) == x
                R._libc.free(ctypes.c_void_p(q))
                n += 1
            td = (time.perf_counter() - t0) / n
            out.append({"kind": kind, "U": U, "C": len(y), "compress_us": round(tc * 1e6, 2),
                        "decompress_us": round(td * 1e6, 2), "ok": ok})
            print(kind, U, out[-1]["compress_us"], out[-1]["decompress_us"], ok, file=sys.stderr, flush=True)
    print(json.dumps({"lib": os.path.basename(R.LIB_PATH), "zc_seg": os.environ.get("RLE_MI355X_ZC_SEG"),
                      "calls": out}))


if __name__ == "__main__":
    main()
