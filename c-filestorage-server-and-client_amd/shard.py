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


def padded_count(n_global: int, world: int) -> int:
    """Entries every rank contributes to the size all-gather: ceil(n_global / world).  A global batch
    that is not a multiple of the world size leaves the last ranks one buffer short; they pad with
    zero-size entries, which sit at global positions >= n_global (k * world + r with k the last local
    index), after every real buffer, so they add nothing to any real buffer's offset."""
    return (n_global + world - 1) // world


def pad_local(local_sizes: torch.Tensor, n_global: int, world: int) -> torch.Tensor:
    """This rank's sizes padded with zeros to padded_count(n_global, world) entries."""
    m = padded_count(n_global, world)
    n = local_sizes.numel()
    if n == m:
        return local_sizes.contiguous()
    assert n == m - 1 or (n == 0 and m <= 1), f"rank holds {n} of {n_global} buffers over {world} ranks"
    return torch.cat([local_sizes, torch.zeros(m - n, dtype=local_sizes.dtype, device=local_sizes.device)])


def global_offsets(local_sizes: torch.Tensor, world: int, n_global: int = None) -> torch.Tensor:
    """All-gather per-buffer compressed sizes (int64, one per local buffer) and return the exclusive
    scan of all sizes in global order: entry i is the byte offset of global buffer i in the
    concatenated stream (n_global entries).  n_global: the global batch size when it is not
    world x the local count (ragged shards, padded by pad_local; default: every rank holds the same
    count).  Collective: every rank must call it."""
    n = local_sizes.numel()
    if n_global is None:
        n_global = n * world
    if world == 1:
        return torch.cumsum(local_sizes, 0) - local_sizes
    padded = pad_local(local_sizes, n_global, world)
    m = padded.numel()
    gathered = torch.empty(world * m, dtype=local_sizes.dtype, device=local_sizes.device)
    dist.all_gather_into_tensor(gathered, padded)
    glob = gathered.view(world, m).t().reshape(-1)[:n_global]   # global order: i = k * world + r
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
    rank's communicator came up (then callers use global_offsets).

    Order of the collective setup, so that no rank can be left waiting in the blocking
    communicator init for a rank that never enters it:
      1. preflight: every rank resolves RCCL (rle_dist_available) and the flags are all-reduced
         with MIN; if any rank failed, no rank goes further;
      2. rank 0 creates the communicator id, broadcast over the process group;
      3. every rank inits its communicator; the result flags are all-reduced with MIN again."""

    def __init__(self, n: int, world: int, rank: int, dev):
        import rle_mi355x as R
        self.R, self.n, self.world, self.ok = R, n, world, False
        self.error = None
        try:
            R.dist_available()
            avail = 1
        except Exception as e:
            avail, self.error = 0, e
        t = torch.tensor([avail], dtype=torch.int32, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        if not t.item():
            if self.error is None:
                self.error = RuntimeError("RCCL unavailable on another rank")
            return
        try:
            uid = [R.dist_unique_id() if rank == 0 else None]
        except Exception as e:   # every rank learns it from the broadcast
            uid, self.error = [None], e
        dist.broadcast_object_list(uid, src=0)
        up = 0
        if uid[0] is not None:
            try:
                R.dist_init(uid[0], rank, world)
                up = 1
            except Exception as e:
                self.error = e
        t = torch.tensor([up], dtype=torch.int32, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        self.ok = bool(t.item())
        if not self.ok:
            if up:
                R.dist_finalize()
            return
        # two result buffers: the exchange of step i may still run (a graph branch) while step i + 1's
        # is issued
        self.gathered = [torch.empty(world * n, dtype=torch.int64, device=dev) for _ in range(2)]
        self.offsets = [torch.empty(world * n, dtype=torch.int64, device=dev) for _ in range(2)]
        # one scan workspace per slot: the two slots' exchanges may run at once (async / graph modes)
        self.ws = [R.dist_workspace(n, dev) for _ in range(2)]

    def step(self, local_sizes: torch.Tensor, stream, slot: int = 0) -> torch.Tensor:
        """Issue one exchange on `stream` after the work issued on it so far, into result buffer
        `slot` (0 or 1); returns the offsets tensor (complete in stream order).  Ragged shards pass
        their sizes padded with zeros to n = padded_count(n_global, world) (pad_local): the result's
        first n_global entries are the offsets of the real buffers."""
        self.R.dist_gather_offsets(local_sizes, self.gathered[slot], self.offsets[slot], stream, ws=self.ws[slot])
        return self.offsets[slot]

    def step_async(self, local_sizes: torch.Tensor, codec_stream, comm_stream, slot: int) -> torch.Tensor:
        """The same exchange on comm_stream, ordered after the work issued on codec_stream so far;
        codec_stream waits only for the previous call's exchange (rle_dist_gather_offsets_async).
        Callers alternate slot 0 / 1 per step."""
        self.R.dist_gather_offsets_async(local_sizes, self.gathered[slot], self.offsets[slot], codec_stream,
                                         comm_stream, slot, ws=self.ws[slot])
        return self.offsets[slot]

    def close(self):
        if self.ok:
            self.R.dist_finalize()
            self.ok = False
