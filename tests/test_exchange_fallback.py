"""CPU multi-process tests (gloo, world size 2) of shard.NativeExchange's collective setup order
(VERDICT r3 item 7): when RCCL cannot be resolved on one rank, or one rank's communicator fails to
come up, EVERY rank must leave the constructor with ok == False -- none may be left waiting in the
blocking communicator init for a rank that never enters it -- and the callers then take the torch
exchange (bench.Exchange mode "torch").  The codec library is replaced by a stub module in each
worker, so no GPU and no RCCL are involved; the process-group traffic (all_reduce, broadcast) is
real gloo traffic."""
import os
import socket
import sys
import types

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _stub(rank, fail_avail_rank, fail_init_rank, calls):
    """A stand-in for rle_mi355x's dist entry points that records which ones each rank reached."""
    m = types.ModuleType("rle_mi355x")

    def dist_available():
        calls.append("available")
        if rank == fail_avail_rank:
            raise OSError("RCCL could not be resolved (test)")

    def dist_unique_id():
        calls.append("unique_id")
        return b"\x01" * 128

    def dist_init(uid, r, w):
        calls.append("init")
        assert uid == b"\x01" * 128 and r == rank
        if rank == fail_init_rank:
            raise RuntimeError("ncclCommInitRank failed (test)")

    def dist_finalize():
        calls.append("finalize")

    def dist_workspace(n, device):
        return torch.empty(1, dtype=torch.int64, device=device)

    m.dist_available, m.dist_unique_id, m.dist_init, m.dist_finalize = (dist_available, dist_unique_id, dist_init,
                                                                       dist_finalize)
    m.dist_workspace = dist_workspace
    return m


def _worker(rank, world, port, fail_avail_rank, fail_init_rank, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    calls = []
    sys.modules["rle_mi355x"] = _stub(rank, fail_avail_rank, fail_init_rank, calls)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        x = shard.NativeExchange(8, world, rank, torch.device("cpu"))
        # the torch exchange the callers fall back to must still work on every rank
        sizes = torch.arange(8, dtype=torch.int64) + 100 * rank
        glob = shard.global_offsets(sizes, world)
        q.put((rank, x.ok, type(x.error).__name__ if x.error is not None else None, calls, glob.tolist()))
    except BaseException as e:   # report instead of leaving the parent waiting on the queue
        q.put((rank, "raised", repr(e), calls, None))
        raise
    finally:
        dist.destroy_process_group()


def _run(fail_avail_rank, fail_init_rank, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fail_avail_rank, fail_init_rank, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, ok, err, calls, glob = q.get(timeout=120)   # a rank stuck in the setup fails the test here
        assert ok != "raised", (rank, err, calls)
        res[rank] = (ok, err, calls, glob)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("bad", [0, 1])
def test_rccl_unavailable_on_one_rank(bad):
    res = _run(fail_avail_rank=bad, fail_init_rank=-1)
    for rank, (ok, err, calls, glob) in res.items():
        assert ok is False
        assert err is not None
        # the preflight stops every rank before the communicator id and the blocking init
        assert calls == ["available"], (rank, calls)
    assert res[0][3] == res[1][3]


def test_init_fails_on_one_rank():
    res = _run(fail_avail_rank=-1, fail_init_rank=1)
    ok0, _, calls0, _ = res[0]
    ok1, err1, calls1, _ = res[1]
    assert ok0 is False and ok1 is False
    assert err1 == "RuntimeError"
    assert calls0 == ["available", "unique_id", "init", "finalize"]   # rank 0's communicator came up: released
    assert calls1 == ["available", "init"]


def test_all_ranks_up():
    res = _run(fail_avail_rank=-1, fail_init_rank=-1)
    for rank, (ok, err, calls, _) in res.items():
        assert ok is True and err is None
        assert calls == (["available", "unique_id", "init"] if rank == 0 else ["available", "init"])
