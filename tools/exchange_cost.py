#!/usr/bin/env python3
"""Host cost of bench.py's N > 1 exchange step (sizes copied, all-gathered over RCCL, scanned into
global offsets) measured on one GPU with a one-rank RCCL process group (the same host call path as
N > 1; the collective itself is trivial).  Compares the enqueue time per step of the codec alone,
the codec plus the current exchange, and the codec plus the exchange variants.
usage: python tools/exchange_cost.py [--steps 200]"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "c-filestorage-server-and-client_amd")]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402
import rle_mi355x as R  # noqa: E402
import shard  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=200)
a = ap.parse_args()
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
s = torch.cuda.current_stream()
comm = torch.cuda.Stream(device=dev)
B = bench.Batch(bench.WORKLOADS["cfg1"], 0, 1, dev)
B.encode(s)
B.calibrate()
sizes = [torch.empty_like(B.clen) for _ in range(2)]
ev = [torch.cuda.Event() for _ in range(2)]


def gather_offsets(x, world):   # shard.global_offsets without its world == 1 shortcut
    n = x.numel()
    g = torch.empty(world * n, dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(g, x.contiguous())
    glob = g.view(world, n).t().reshape(-1)
    return torch.cumsum(glob, 0) - glob


def run(name, fn):
    for _ in range(20):
        fn(0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        fn(i)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{name}: enqueue {(t1 - t0) / a.steps * 1e6:.1f} us/step, wall {(t2 - t0) / a.steps * 1e6:.1f} us/step")


def codec(i):
    B.encode(s)
    B.decode(s)


def current(i):
    B.encode(s)
    k = i % 2
    s.wait_event(ev[k])
    sizes[k].copy_(B.clen)
    comm.wait_stream(s)
    with torch.cuda.stream(comm):
        gather_offsets(sizes[k], 1)
        ev[k].record(comm)
    B.decode(s)


g_pre = torch.empty(B.n, dtype=torch.int64, device=dev)


def only_copy(i):
    codec(i)
    sizes[i % 2].copy_(B.clen)


def only_gather(i):
    codec(i)
    dist.all_gather_into_tensor(g_pre, sizes[0])


def only_scan(i):
    codec(i)
    glob = g_pre.view(1, B.n).t().reshape(-1)
    torch.cumsum(glob, 0) - glob


def only_streams(i):
    codec(i)
    k = i % 2
    s.wait_event(ev[k])
    comm.wait_stream(s)
    with torch.cuda.stream(comm):
        ev[k].record(comm)


run("codec only", codec)
run("codec + copy_", only_copy)
run("codec + all_gather_into_tensor", only_gather)
run("codec + view/t/reshape/cumsum/sub", only_scan)
run("codec + stream waits and event", only_streams)
run("codec + exchange as torch calls (bench.py before rle_dist)", current)
nx = shard.NativeExchange(B.n, 1, 0, dev)
print("native exchange up:", nx.ok, nx.error)


def native(i):
    B.encode(s)
    nx.step(B.clen, s)
    B.decode(s)


if nx.ok:
    run("codec + native exchange (rle_dist_gather_offsets, same stream)", native)

    def gather_only(i):
        B.encode(s)
        dist.all_gather_into_tensor(nx.gathered, B.clen)
        B.decode(s)

    run("codec + torch all_gather_into_tensor only, same stream", gather_only)
    torch.cuda.synchronize()
    ref = torch.cumsum(B.clen, 0) - B.clen
    print("native offsets match cumsum:", bool(torch.equal(nx.offsets, ref)))
    nx.close()
print("shard.global_offsets is", shard.global_offsets)
dist.destroy_process_group()
