"""Position-level model of the decode kernel's LDS staging (csrc/rle_device.h: dec_tile, dec_flush,
dec_finish), used by tests/test_dec_stage_model.py on CPU.

It restates what one wave does per 1008-byte tile of a well-formed stream (encoder output: every
3-byte token's count digit in '2'..'9'; the kernel sends anything else to its serial path):
  * token starts and decoded lengths W per position (reference src/rleCompression.c:50-60);
  * the lanes' output offsets, and the split of the tile into passes over consecutive lanes when
    the staging (kDecChunks chunks of 16 u16 keys) cannot hold the tile's output at once;
  * the scatter: a token start writes a flagged key at its decoded position, every other owned
    position writes an unflagged key one slot before its running offset;
  * the flush of complete chunks: each position takes the byte of the latest flagged key at or
    before it in its chunk, else the carry (the last byte of the chunk before); chunks are zeroed,
    and the partial chunk moves to chunk 1.
Slots are 16 + (decoded position - flushed); chunk 0 is the guard.  Writes past the staging raise,
so the test also checks the pass split's capacity bound.
"""

TILE = 1008     # kTileStep: 63 owned lanes x 16 positions
LANES = 63
FLAG = 0x8000


def decode_staged(y: bytes, U: int, chunks: int):
    """Decode stream y (length C) to U bytes through a staging of `chunks` chunks per wave.
    Returns (output bytes, number of passes per tile)."""
    C = len(y)
    cap = 16 * chunks - 17                  # kDecPassCap
    one_pass = chunks >= 191                # kDecOnePass
    # token parse over the whole stream: W[p] = decoded bytes of a token starting at p, else 0
    W = [0] * C
    start = [False] * C
    p = 0
    while p < C:
        start[p] = True
        if p + 1 < C and y[p] == y[p + 1]:
            d = y[p + 2] - ord("0")
            assert 2 <= d <= 9, "not an encoder stream (the kernel would take its serial path)"
            W[p] = d
            p += 3
        else:
            W[p] = 1
            p += 1
    stage = [0] * (16 * chunks)
    out = bytearray()
    out_pos = flushed = 0
    fillc = 0
    passes = []

    # The 63 lanes write in parallel (16 ds_write_b16 each), so the model collects one pass's writes
    # and rejects any slot that receives a flagged key together with any other write: the result
    # would depend on the order of the lanes' stores.
    writes = {}

    def put(idx, key):
        if not 15 <= idx < len(stage):
            raise IndexError(f"staging write at slot {idx} outside [15, {len(stage)})")
        writes.setdefault(idx, []).append(key)

    def commit():
        for idx, keys in writes.items():
            if len(keys) > 1 and any(k & FLAG for k in keys):
                raise AssertionError(f"slot {idx}: a flagged key and another write in one pass")
            stage[idx] = keys[-1]
        writes.clear()

    def fill_chunk(keys, carry):
        cur, res = carry, bytearray()
        for k in keys:
            if k & FLAG:
                cur = k & 0xFF
            res.append(cur)
        return res

    for t0 in range(0, C, TILE):
        # lane output counts and inclusive offsets within the tile
        nout = [sum(W[q] for q in range(t0 + 16 * l, min(t0 + 16 * l + 16, C))) for l in range(LANES)]
        oincl, s = [], 0
        for n in nout:
            s += n
            oincl.append(s)
        ttot = s
        done = frm = 0
        npass = 0
        while True:
            rel0 = out_pos + done - flushed
            assert 0 <= rel0 < 16
            upto, pss = LANES, ttot - done
            if not one_pass and rel0 + pss > cap:
                fit = [l for l in range(LANES) if oincl[l] <= done + cap - rel0]
                upto = len(fit)
                assert fit == list(range(upto)) and upto > frm, "pass split must be a prefix that progresses"
                pss = oincl[upto - 1] - done
            assert rel0 + pss <= cap or one_pass
            for l in range(frm, upto):
                off = oincl[l] - nout[l] - done          # lane's output start, relative to the pass
                for q in range(t0 + 16 * l, min(t0 + 16 * l + 16, C)):
                    if start[q]:
                        put(16 + rel0 + off, FLAG | y[q])
                    else:
                        put(16 + rel0 + off - 1, y[q])  # one slot back: its token's last position
                    off += W[q]
            commit()
            newrel = rel0 + pss
            nfl = newrel >> 4
            for c in range(1, nfl + 1):
                keys = stage[16 * c:16 * c + 16]
                chunk = fill_chunk(keys, fillc)
                out += chunk
                fillc = chunk[-1]
                stage[16 * c:16 * c + 16] = [0] * 16
            if nfl:
                stage[16:32] = stage[16 * (nfl + 1):16 * (nfl + 2)]
                stage[16 * (nfl + 1):16 * (nfl + 2)] = [0] * 16
            flushed += 16 * nfl
            done += pss
            frm = upto
            npass += 1
            if upto >= LANES:
                break
        out_pos += ttot
        passes.append(npass)
    # dec_finish: the staged partial chunk, then zeros up to U
    rel = out_pos - flushed
    out += fill_chunk(stage[16:16 + rel], fillc)
    out += bytes(max(0, U - len(out)))
    return bytes(out[:U]), passes
