"""GPU tests of the multi-GPU exchange (csrc/rle_dist.hip): the reorder + exclusive
scan into global stream order against numpy at several world sizes, and one whole exchange step
through a one-rank RCCL communicator (the only size one GPU can run; the N-rank path is the same
calls)."""
import numpy as np
import pytest
import torch

import rle_mi355x as R

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _ref_offsets(gathered, world, n):
    glob = gathered.reshape(world, n).T.reshape(-1)   # global i = k * world + r
    return np.cumsum(glob) - glob


@pytest.mark.parametrize("world,n", [(1, 1), (2, 7), (3, 1000), (8, 4096), (8, 131072), (1, 1 << 20),
                                     (5, 300000), (16, 65537), (17, 1000),
                                     # just past the one-workgroup form (n <= 512), and around 8192
                                     (1, 513), (8, 1025), (2, 8191), (16, 8192), (3, 8193)])
def test_offsets_kernel_global_order(world, n):
    rng = np.random.default_rng(world * 1000 + n)
    g = rng.integers(0, 70000, size=world * n, dtype=np.int64)
    d_g = torch.from_numpy(g).to(DEV)
    d_o = torch.full((world * n,), -1, dtype=torch.int64, device=DEV)
    R.dist_offsets(d_g, world, n, d_o)
    torch.cuda.synchronize()
    assert np.array_equal(d_o.cpu().numpy(), _ref_offsets(g, world, n))


def test_exchange_step_one_rank():
    uid = R.dist_unique_id()
    R.dist_init(uid, 0, 1)
    try:
        n = 4096
        sizes = torch.randint(1, 6000, (n,), dtype=torch.int64, device=DEV)
        gathered = torch.empty_like(sizes)
        offsets = torch.full((n,), -1, dtype=torch.int64, device=DEV)
        s = torch.cuda.current_stream()
        for _ in range(3):   # repeated steps reuse the buffers
            R.dist_gather_offsets(sizes, gathered, offsets, s)
        torch.cuda.synchronize()
        assert torch.equal(gathered, sizes)
        assert torch.equal(offsets, torch.cumsum(sizes, 0) - sizes)
    finally:
        R.dist_finalize()


@pytest.mark.parametrize("world,n_global", [(3, 1000), (8, 131071), (2, 4097)])
def test_offsets_kernel_ragged_padded(world, n_global):
    """Ragged shards (shard.pad_local): each rank's sizes padded with zeros to ceil(n_global / world);
    the reorder + scan kernel over the padded all-gather gives, in its first n_global entries, the
    single-process exclusive scan of the real sizes."""
    import shard
    rng = np.random.default_rng(n_global)
    sizes = rng.integers(0, 70000, size=n_global, dtype=np.int64)
    m = shard.padded_count(n_global, world)
    rows = [shard.pad_local(torch.from_numpy(sizes[r::world].copy()), n_global, world).numpy() for r in range(world)]
    g = np.concatenate(rows)
    d_g = torch.from_numpy(g).to(DEV)
    d_o = torch.full((world * m,), -1, dtype=torch.int64, device=DEV)
    R.dist_offsets(d_g, world, m, d_o)
    torch.cuda.synchronize()
    assert np.array_equal(d_o.cpu().numpy()[:n_global], np.cumsum(sizes) - sizes)


def test_exchange_step_one_rank_padded_count():
    """The one-rank RCCL rehearsal with a padded count: zero-size entries past the real buffers
    leave every real offset equal to the cumsum of the real sizes."""
    uid = R.dist_unique_id()
    R.dist_init(uid, 0, 1)
    try:
        n_real, n = 4093, 4096
        sizes = torch.randint(1, 6000, (n,), dtype=torch.int64, device=DEV)
        sizes[n_real:] = 0
        gathered = torch.empty_like(sizes)
        offsets = torch.full((n,), -1, dtype=torch.int64, device=DEV)
        R.dist_gather_offsets(sizes, gathered, offsets, torch.cuda.current_stream())
        torch.cuda.synchronize()
        real = sizes[:n_real]
        assert torch.equal(offsets[:n_real], torch.cumsum(real, 0) - real)
    finally:
        R.dist_finalize()


def test_exchange_captured_in_graph_one_rank():
    """The graph form bench.py uses at N > 1: the exchange issued on a branch stream inside a HIP
    graph capture (fork / join by events), replayed several times, gives the same offsets."""
    uid = R.dist_unique_id()
    R.dist_init(uid, 0, 1)
    try:
        n = 4096
        sizes = torch.randint(1, 6000, (n,), dtype=torch.int64, device=DEV)
        gathered = torch.empty_like(sizes)
        offsets = torch.full((n,), -1, dtype=torch.int64, device=DEV)
        ws = R.dist_workspace(n, DEV)   # the caller's: alive as long as the graph
        R.dist_gather_offsets(sizes, gathered, offsets, ws=ws)
        torch.cuda.synchronize()
        offsets.fill_(-1)
        g = torch.cuda.CUDAGraph()
        main, side = torch.cuda.Stream(), torch.cuda.Stream()
        main.wait_stream(torch.cuda.current_stream())
        with torch.cuda.graph(g, stream=main, capture_error_mode="relaxed"):
            side.wait_stream(main)
            R.dist_gather_offsets(sizes, gathered, offsets, side, ws=ws)
            main.wait_stream(side)
        torch.cuda.synchronize()
        for _ in range(3):
            offsets.fill_(-1)
            g.replay()
            torch.cuda.synchronize()
            assert torch.equal(offsets, torch.cumsum(sizes, 0) - sizes)
        del g
    finally:
        R.dist_finalize()


@pytest.mark.parametrize("xmode", ["async", "inline", "graph", "auto"])
def test_bench_exchange_path_one_rank(xmode):
    """bench.py's N > 1 rank loop rehearsed on one GPU (RLE_BENCH_FORCE_EXCHANGE=1): a one-rank
    process group over RCCL, the native exchange in each mode (side stream, codec stream, captured
    with the timed loop in one HIP graph, and the default: inline and async timed, the faster
    kept), the offsets checked against the process-group path, and the round trip verified."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, RLE_BENCH_FORCE_EXCHANGE="1", RLE_BENCH_XMODE=xmode)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "6", "--warmup", "2", "--no-cpu",
                        "--no-north-star", "--no-concurrent"], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["verified_bit_exact_roundtrip"] is True
    if xmode == "auto":
        t = out["exchange"]["auto_us_per_step"]
        assert set(t) == {"inline", "async"} and out["exchange"]["mode"] == min(t, key=t.get), out["exchange"]
    else:
        assert out["exchange"]["mode"] == xmode, out["exchange"]
    assert out["exchange"]["graph_captured"] is (True if xmode == "graph" else None)
    assert out["exchange"]["offsets_match_process_group"] is True


def test_exchange_async_alternating_slots():
    """rle_dist_gather_offsets_async over several steps with the sizes rewritten every step (the
    bench's pattern: slot i % 2): every step's offsets are that step's scan."""
    uid = R.dist_unique_id()
    R.dist_init(uid, 0, 1)
    try:
        n = 4096
        codec, comm = torch.cuda.current_stream(), torch.cuda.Stream()
        sizes = [torch.zeros(n, dtype=torch.int64, device=DEV) for _ in range(2)]
        gathered = [torch.empty(n, dtype=torch.int64, device=DEV) for _ in range(2)]
        offsets = [torch.empty(n, dtype=torch.int64, device=DEV) for _ in range(2)]
        ws = [R.dist_workspace(n, DEV) for _ in range(2)]
        want = []
        for i in range(6):
            s = i % 2
            v = torch.randint(1, 6000, (n,), dtype=torch.int64, device=DEV)
            sizes[s].copy_(v)   # the "encode" of step i, on the codec stream
            R.dist_gather_offsets_async(sizes[s], gathered[s], offsets[s], codec, comm, s, ws=ws[s])
            want.append(torch.cumsum(v, 0) - v)
            if i >= 4:
                torch.cuda.synchronize()
                assert torch.equal(offsets[s], want[i])
    finally:
        torch.cuda.synchronize()
        R.dist_finalize()


def test_exchange_async_repeated_slot_refused():
    """A slot repeated while its previous exchange is still queued would let the codec stream wait
    on the stale other slot: refused.  Once that exchange has completed (a warm-up
    before the timed loop, bench.py), the repeat is accepted."""
    uid = R.dist_unique_id()
    R.dist_init(uid, 0, 1)
    try:
        n = 1024
        codec, comm = torch.cuda.current_stream(), torch.cuda.Stream()
        sizes = torch.ones(n, dtype=torch.int64, device=DEV)
        g = torch.empty(n, dtype=torch.int64, device=DEV)
        o = torch.empty(n, dtype=torch.int64, device=DEV)
        big = torch.empty(1 << 30, dtype=torch.uint8, device=DEV)
        with torch.cuda.stream(comm):   # keeps the first exchange queued for a few ms
            for _ in range(8):
                big.fill_(1)
        R.dist_gather_offsets_async(sizes, g, o, codec, comm, 0)
        with pytest.raises(R.RLEError):
            R.dist_gather_offsets_async(sizes, g, o, codec, comm, 0)
        R.dist_gather_offsets_async(sizes, g, o, codec, comm, 1)
        torch.cuda.synchronize()
        assert torch.equal(o, torch.arange(n, dtype=torch.int64, device=DEV))
        R.dist_gather_offsets_async(sizes, g, o, codec, comm, 1)   # slot 1 again: its exchange is done
        torch.cuda.synchronize()
        assert torch.equal(o, torch.arange(n, dtype=torch.int64, device=DEV))
    finally:
        torch.cuda.synchronize()
        R.dist_finalize()


def test_offsets_two_streams_own_workspaces():
    """Two whole-chip scans (n > 512) queued at once on two streams, each with its own workspace
    (the process-wide workspace let them overwrite each other's tile sums)."""
    world, n = 8, 131072
    rng = np.random.default_rng(7)
    gs = [rng.integers(0, 70000, size=world * n, dtype=np.int64) for _ in range(2)]
    d_g = [torch.from_numpy(g).to(DEV) for g in gs]
    d_o = [torch.full((world * n,), -1, dtype=torch.int64, device=DEV) for _ in range(2)]
    ws = [R.dist_workspace(n, DEV) for _ in range(2)]
    st = [torch.cuda.Stream(), torch.cuda.Stream()]
    torch.cuda.synchronize()
    for rep in range(5):
        for k in range(2):
            R.dist_offsets(d_g[k], world, n, d_o[k], st[k], ws=ws[k])
    torch.cuda.synchronize()
    for k in range(2):
        assert np.array_equal(d_o[k].cpu().numpy(), _ref_offsets(gs[k], world, n))
