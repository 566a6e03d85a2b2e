"""CPU multi-process tests of the N > 1 path (gloo, world size 2): round-robin sharding and the
size all-gather + global-order scan reproduce the single-process layout of the compressed
stream exactly (the oracle stands in for the per-rank codec here)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import shard
import rle_oracle as O


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_global, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        idx = shard.shard_indices(n_global, rank, world)
        assert len(idx) == shard.local_count(n_global, rank, world)
        streams = {}
        sizes = []
        for i in idx:
            x = O.gen(i % 5, i, 1000 + (i * 37) % 3000)
            y = O.encode(x)
            streams[i] = y
            sizes.append(len(y))
        ragged = n_global % world != 0
        glob = shard.global_offsets(torch.tensor(sizes, dtype=torch.int64), world,
                                    n_global=n_global if ragged else None)
        mine = shard.my_offsets(glob, rank, world)
        q.put((rank, {i: (int(o), s) for i, o, s in zip(idx, mine.tolist(), [streams[i] for i in idx])},
               glob.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_global", [(2, 64), (3, 1000), (2, 63), (3, 2)])
def test_round_robin_shards_and_global_offsets(world, n_global):
    """Equal shards (64 over 2) and ragged ones (1000 over 3, 63 over 2, 2 over 3: a rank with no
    buffer), each rank's sizes padded with zeros to ceil(n_global / world) for the all-gather."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_global, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single-process reference layout
    ref = [O.encode(O.gen(i % 5, i, 1000 + (i * 37) % 3000)) for i in range(n_global)]
    ref_off = np.concatenate([[0], np.cumsum([len(y) for y in ref])[:-1]])
    whole = b"".join(ref)
    globs = [g for _, _, g in res]
    assert all(g == globs[0] for g in globs)
    assert globs[0] == ref_off.tolist()
    # each rank's streams, placed at its global offsets, rebuild the single-process stream
    buf = bytearray(len(whole))
    seen = set()
    for _, d, _ in res:
        for i, (off, y) in d.items():
            buf[off:off + len(y)] = y
            seen.add(i)
    assert seen == set(range(n_global))
    assert bytes(buf) == whole


def test_shard_indices_cover_once():
    for world in (1, 2, 3, 8):
        n = 1000
        allidx = sorted(i for r in range(world) for i in shard.shard_indices(n, r, world))
        assert allidx == list(range(n))
        assert sum(shard.local_count(n, r, world) for r in range(world)) == n


def test_padding_rule_matches_single_process_cumsum():
    """The padded all-gather's layout (no processes): every rank's sizes padded to ceil(n / world),
    interleaved in global order and cut at n, equals the single-process exclusive scan."""
    rng = np.random.default_rng(3)
    for world in (1, 2, 3, 7, 8):
        for n in (1, 2, 7, 8, 9, 1000, 1001, 1023):
            sizes = rng.integers(0, 100000, size=n)
            m = shard.padded_count(n, world)
            rows = []
            for r in range(world):
                loc = torch.tensor(sizes[r::world], dtype=torch.int64)
                assert loc.numel() == shard.local_count(n, r, world)
                rows.append(shard.pad_local(loc, n, world))
            gathered = torch.stack(rows)              # [world, m], as all_gather_into_tensor lays it out
            glob = gathered.t().reshape(-1)[:n]
            assert glob.numel() == n and m * world - n < world
            off = (torch.cumsum(glob, 0) - glob).numpy()
            assert np.array_equal(off, np.cumsum(sizes) - sizes), (world, n)
