"""CPU model of the large decode batches' issue order (csrc/rle_kernels.hip dec_order_local_kernel and
order_slot_local, round 5): each chunk of 256 buffers is sorted by descending tile count in its
workgroup, and the decode kernel's issue slot s takes place s // F of chunk s % F (F full chunks), the
partial last chunk after them.  Pins that every buffer is issued exactly once for any batch size, and
that on batches whose chunks hold the same mix the interleaved order is the global longest-first order
up to ties."""
import numpy as np
import pytest

CHUNK = 256          # kLocalChunk
TILE = 1008          # kTileStep
BUCKETS = 2048       # kOrderBuckets


def order_key(c):
    t = (c + TILE - 1) // TILE
    return min(t, BUCKETS - 1)


def local_order(lengths):
    """order[] as dec_order_local_kernel writes it: chunk by chunk, longest first inside a chunk (a
    bucket's members in any order: here by index, as one valid outcome of the LDS atomics)."""
    n = len(lengths)
    order = np.empty(n, dtype=np.int64)
    for c0 in range(0, n, CHUNK):
        idx = np.arange(c0, min(n, c0 + CHUNK))
        keys = np.array([order_key(int(lengths[i])) for i in idx])
        order[c0:c0 + len(idx)] = idx[np.argsort(-keys, kind="stable")]
    return order


def slot_to_place(s, n):
    F = n // CHUNK
    if s >= F * CHUNK:
        return s
    return (s % F) * CHUNK + s // F


@pytest.mark.parametrize("n", [4097, 4099, 5000, 8195, 12288, 16384, 16385, 65536, 65537])
def test_every_buffer_issued_once(n):
    rng = np.random.default_rng(n)
    lengths = rng.integers(0, 70000, size=n)
    order = local_order(lengths)
    issued = np.array([order[slot_to_place(s, n)] for s in range(n)])
    assert np.array_equal(np.sort(issued), np.arange(n))


def test_interleaved_chunks_are_longest_first_on_uniform_mixes():
    # dec64k's shape: buffer i of kind i % 4 (zero / random / runs50 / runs90 compress to about 22,
    # 66, 66 and 30 tiles), 16384 buffers
    n = 16384
    tiles = np.array([22, 66, 65, 30])
    lengths = np.array([tiles[i % 4] * TILE - 5 for i in range(n)])
    order = local_order(lengths)
    keys = np.array([order_key(int(lengths[order[slot_to_place(s, n)]])) for s in range(n)])
    assert np.all(np.diff(keys) <= 0), "the issue order is not longest first"


XCDS = 8
DEC_WAVES = 4        # RLE_DEC_WAVES


def grid_for(n, waves=DEC_WAVES):
    g = (n + waves - 1) // waves
    return (g + XCDS - 1) // XCDS * XCDS

