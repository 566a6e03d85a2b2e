#!/usr/bin/env python3
"""Markdown table of a tools/ab_events.py run (its stdout): per workload, each build's median
encode / decode µs and the decode change against the product build, plus the round-trip check.
usage: python tools/ab_events_table.py gpurun_out/<tag>/ab.json [title]"""
import json
import sys


def main():
    path = sys.argv[1]
    title = sys.argv[2] if len(sys.argv) > 2 else path
    rows = []
    for line in open(path):
        line = line.strip()
        if not line or line.startswith("{"):
            continue
        wl, js = line.split(" ", 1)
        rows.append((wl, json.loads(js)))
    builds = list(rows[0][1]) if rows else []
    print(f"# {title}\n")
    print("Same-process A/B (tools/ab_events.py): median of the rounds, each round the mean of back-to-back "
          "launches timed by HIP events.  ok = the build's round trip reproduced the input exactly "
          "(ablation builds are timing-only and may fail it).\n")
    print("| workload | build | encode µs | decode µs | decode vs product | ok |")
    print("|---|---|---|---|---|---|")
    for wl, d in rows:
        base = d["product"]["dec"]["median_us"]
        for b in builds:
            v = d[b]
            dec = v["dec"]["median_us"]
            print(f"| {wl} | {b} | {v['enc']['median_us']:.2f} | {dec:.2f} | {100 * (dec / base - 1):+.1f} % | "
                  f"{'yes' if v['ok'] else 'no'} |")


if __name__ == "__main__":
    main()
