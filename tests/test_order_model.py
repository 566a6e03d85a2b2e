"""CPU model of the large decode batches' issue order (csrc/rle_kernels.hip dec_order_local_kernel and
order_slot_local, round 5): each chunk of 256 buffers is sorted by descending tile count in its
workgroup, and the decode kernel's issue slot s takes place s // F of chunk s % F (F full chunks), the
partial last chunk after them.  Pins that every buffer is issued exactly once for any batch size, and
that on batches whose chunks hold the same mix the interleaved order is the global longest-first order
up to ties."""
import numpy as np
import pytest

CHUNK = 256          # kLocalChunk (256 x RLE_ORDER_LOCAL_PER = 1)
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


def order_place_xcd(wg, ngrid, wid, n):
    """csrc/rle_kernels.hip order_place_xcd (RLE_ORDER_XCD=1)."""
    R = ngrid // XCDS * DEC_WAVES
    a = (wg % XCDS) * R
    k = (wg // XCDS) * DEC_WAVES + wid
    if a >= n or k >= n - a:
        return n
    L = min(n - a, R)
    c0, c1 = (a + CHUNK - 1) // CHUNK, (a + L) // CHUNK
    F = max(c1 - c0, 0)
    if k < F * CHUNK:
        return (c0 + k % F) * CHUNK + k // F
    if F == 0:
        return a + k
    r, h = k - F * CHUNK, c0 * CHUNK - a
    return a + r if r < h else c1 * CHUNK + (r - h)


@pytest.mark.parametrize("n", [1, 7, 255, 4097, 4099, 5000, 8195, 12288, 16384, 16385, 65536, 65537, 100003])
def test_xcd_places_cover_the_batch_once(n):
    g = grid_for(n)
    places = [order_place_xcd(wg, g, w, n) for wg in range(g) for w in range(DEC_WAVES)]
    got = np.sort(np.array([p for p in places if p < n]))
    assert np.array_equal(got, np.arange(n))


def test_xcd_slices_are_longest_first_on_uniform_mixes():
    n = 16384
    tiles = np.array([22, 66, 65, 30])
    lengths = np.array([tiles[i % 4] * TILE - 5 for i in range(n)])
    order = local_order(lengths)
    g = grid_for(n)
    for x in range(XCDS):
        wgs = range(x, g, XCDS)
        places = [order_place_xcd(wg, g, w, n) for wg in wgs for w in range(DEC_WAVES)]
        assert min(places) >= x * n // XCDS and max(places) < (x + 1) * n // XCDS
        keys = np.array([order_key(int(lengths[order[p]])) for p in places])
        assert np.all(np.diff(keys) <= 0), f"XCD {x} does not walk its slice longest first"


def slot_to_place_grouped(s, n, G):
    """order_slot_local with RLE_ORDER_GROUP = G."""
    F = n // CHUNK
    if s >= F * CHUNK:
        return s
    q = s // G
    return (q % F) * CHUNK + (q // F) * G + s % G


@pytest.mark.parametrize("G", [1, 4, 8])
@pytest.mark.parametrize("n", [4097, 8195, 16384, 65537])
def test_grouped_slots_cover_the_batch_once(n, G):
    places = np.array([slot_to_place_grouped(s, n, G) for s in range(n)])
    assert np.array_equal(np.sort(places), np.arange(n))
    if G == 1:
        assert all(slot_to_place(s, n) == places[s] for s in range(0, n, 97))
