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


@pytest.mark.parametrize("world,n", [(1, 1), (2, 7), (3, 1000), (8, 4096), (8, 131072)])
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
