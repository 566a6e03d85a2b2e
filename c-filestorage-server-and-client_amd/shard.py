"""Sharding of a batch of independent buffers across the GPUs of one node.

Every buffer of the reference codec is independent (src/rleCompression.c keeps no state across
calls), so a global batch shards with no data-path collective: buffer i goes to rank i % N
(round-robin) and is encoded, stored and decoded on that GPU.  The one exchange step is the
all-gather of the per-buffer compressed sizes (u64), after which every rank can place any
buffer's compressed stream in the global, buffer-ordered stream (an exclusive scan in global
order).  With the NCCL backend torch.distributed runs this over RCCL / xGMI; the payloads stay
where they are.
"""
import torch
import torch.distributed as dist


def shard_indices(n_global: int, rank: int, world: int):
    """Global buffer indices owned by `rank` (round-robin: i % world == rank), in local order."""
    return list(range(rank, n_global, world))


def local_count(n_global: int, rank: int, world: int) -> int:
    return (n_global - rank + world - 1) // world if rank < n_global else 0


def global_offsets(local_sizes: torch.Tensor, world: int) -> torch.Tensor:
    """All-gather per-buffer compressed sizes (int64, one per local buffer, every rank holding the
    same count) and return the exclusive scan of all sizes in global order: entry i is the byte
    offset of global buffer i in the concatenated stream.  Collective: every rank must call it."""
    n = local_sizes.numel()
    if world == 1:
        return torch.cumsum(local_sizes, 0) - local_sizes
    gathered = torch.empty(world * n, dtype=local_sizes.dtype, device=local_sizes.device)
    dist.all_gather_into_tensor(gathered, local_sizes.contiguous())
    glob = gathered.view(world, n).t().reshape(-1)   # global order: i = k * world + r
    return torch.cumsum(glob, 0) - glob


def my_offsets(glob_offsets: torch.Tensor, rank: int, world: int) -> torch.Tensor:
    """This rank's buffers' offsets in the global stream."""
    return glob_offsets[rank::world]


class NativeExchange:
    """global_offsets as one library call per step (rle_dist_gather_offsets, csrc/rle_dist.hip):
    the sizes all-gathered over RCCL and scanned on the codec's stream.  The same exchange issued as
    torch calls on a side stream costs 56-87 us of host time per configs[1] step against ~21 us of
    GPU time (tools/exchange_cost.py).  Collective setup: every rank constructs it; rank 0's
    communicator id is broadcast over the process group.  `ok` is False on every rank unless every
    rank's communicator came up (then callers use global_offsets)."""

    def __init__(self, n: int, world: int, rank: int, dev):
        import rle_mi355x as R
        self.R, self.n, self.world, self.ok = R, n, world, False
        err = None
        try:
            uid = [R.dist_unique_id() if rank == 0 else None]
        except Exception as e:   # no RCCL symbols: every rank learns it below
            uid, err = [None], e
        dist.broadcast_object_list(uid, src=0)
        up = 0
        if uid[0] is not None:
            try:
                R.dist_init(uid[0], rank, world)
                up = 1
            except Exception as e:
                err = e
        t = torch.tensor([up], dtype=torch.int32, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        self.ok = bool(t.item())
        self.error = err
        if not self.ok:
            if up:
                R.dist_finalize()
            return
        self.gathered = torch.empty(world * n, dtype=torch.int64, device=dev)
        self.offsets = torch.empty(world * n, dtype=torch.int64, device=dev)

    def step(self, local_sizes: torch.Tensor, stream) -> torch.Tensor:
        """Issue one exchange on `stream` after the work issued on it so far; returns the offsets
        tensor (complete in stream order)."""
        self.R.dist_gather_offsets(local_sizes, self.gathered, self.offsets, stream)
        return self.offsets

    def close(self):
        if self.ok:
            self.R.dist_finalize()
            self.ok = False
