"""Pure-Python model of the SEGMENTED codec (several waves per buffer): the per-segment summaries
and the per-buffer scan that the HIP kernels enc_seg_* / dec_seg_* implement, written plainly so
tests/test_seg_model.py can check the algebra against the oracle on small inputs.

Encode (reference src/rleCompression.c:9-45; closed form SURVEY.md Appendix A.1).  Segment k
covers input [p0, p1).  A token starts at i iff (i - runstart(i)) mod 9 == 0, so a segment
depends on the data before it only through the phase of the run that enters it:
  summary (local):  L0   = offset of the first run boundary in the segment (p1 - p0 if none)
                    lb   = last boundary position in the segment (None if none)
                    cont = the segment has no boundary and its run continues past p1
                    rest = compressed bytes of the tokens starting at or after p0 + L0
  scan (per buffer): rs_k = last boundary before p0 (a running max of lb), q = run phase of byte
                    p0 - 1; the entering piece [p0, p0 + L0) holds token starts at offsets
                    k0 = (8 - q) mod 9 + 9 m, each 3 bytes except a last byte of the run (1 byte).
Decode (reference src/rleCompression.c:47-62).  Segment k covers stream [q0, q1); the first token
start in it is q0 + e, e in {0,1,2}.  For every e the summary records the exit offset and the
decoded byte count, so segments compose like the in-wave phase maps (v_perm selectors).
"""

SEG_NONE = None


def _bnd(x, i):
    return i == 0 or x[i] != x[i - 1]


def enc_summary(x, p0, p1):
    U = len(x)
    L0 = None
    lb = None
    for i in range(p0, p1):
        if _bnd(x, i):
            if L0 is None:
                L0 = i - p0
            lb = i
    if L0 is None:
        L0 = p1 - p0
    cont = L0 == p1 - p0 and p1 < U and x[p1] == x[p1 - 1]
    # tokens starting at or after the first boundary: plain restatement of A.1
    rest = 0
    i = p0 + L0
    rs = i
    while i < p1:
        if _bnd(x, i):
            rs = i
        if (i - rs) % 9 == 0:
            j = i
            while j + 1 < U and x[j + 1] == x[i] and j + 1 - i < 9:
                j += 1
            rest += 1 if j == i else 3
        i += 1
    return L0, lb, cont, rest


def enc_piece_count(L0, q, cont):
    """compressed bytes of the tokens starting in the entering run piece of length L0, when the
    byte before the segment has run phase q"""
    if L0 == 0:
        return 0
    k0 = (8 - q) % 9
    if L0 <= k0:
        return 0
    n = (L0 - 1 - k0) // 9 + 1
    last_is_start = (L0 - 1 - k0) % 9 == 0
    return 3 * n - (2 if last_is_start and not cont else 0)


def enc_scan(x, segs):
    """segs: list of (p0, p1) covering x in order -> (per segment (rs, off, cnt), total C)"""
    out, off, rs_run = [], 0, 0
    for (p0, p1) in segs:
        L0, lb, cont, rest = enc_summary(x, p0, p1)
        if p0 == 0:
            piece = 0   # position 0 is a boundary, L0 == 0
        else:
            q = (p0 - 1 - rs_run) % 9
            piece = enc_piece_count(L0, q, cont)
        cnt = piece + rest
        out.append((rs_run, off, cnt))
        off += cnt
        if lb is not None:
            rs_run = lb
    return out, off


def enc_write(x, p0, p1, rs):
    """the compressed bytes of the tokens starting in [p0, p1), given the run start rs entering"""
    U = len(x)
    y = bytearray()
    run = rs
    for i in range(p0, p1):
        if _bnd(x, i):
            run = i
        if (i - run) % 9 == 0:
            j = i
            while j + 1 < U and x[j + 1] == x[i] and j + 1 - i < 9:
                j += 1
            r = j - i + 1
            y += bytes([x[i]]) if r == 1 else bytes([x[i], x[i], 48 + r])
    return bytes(y)


def dec_summary(y, q0, q1):
    """for entry offsets e = 0, 1, 2: (exit offset past q1, decoded count, ok).  ok is False where
    the tiled path would decline (count digit outside '1'..'9' with the digit inside the stream);
    a digit read from the padding (the stream's final token) gives 1 byte here and is handled by
    the caller (tail)."""
    C = len(y)
    res = []
    for e in range(3):
        j, cnt, ok = q0 + e, 0, True
        while j < q1:
            v = y[j]
            n1 = y[j + 1] if j + 1 < C else 0
            if v == n1:
                if j + 2 < C:
                    d = y[j + 2]
                    if 0x31 <= d <= 0x39:
                        cnt += d - 48
                    else:
                        ok = False
                        cnt += 1
                else:
                    cnt += 1   # final token: its run extends to U (tail)
                j += 3
            else:
                cnt += 1
                j += 1
        res.append((j - q1, cnt, ok))
    return res


def dec_scan(y, segs):
    """segs: list of (q0, q1) covering y in order -> per segment (entry offset, output offset)"""
    e, off, out, ok = 0, 0, [], True
    for (q0, q1) in segs:
        s = dec_summary(y, q0, q1)
        ex, cnt, good = s[e] if e < 3 else (0, 0, False)
        out.append((e, off))
        ok = ok and good
        off += cnt
        e = ex
    return out, off, ok


def dec_write(y, q0, q1, e, U, off):
    """decode the tokens starting in [q0 + e, q1) into positions [off, ...) (capped at U), the
    final unbounded token filling to U"""
    C = len(y)
    out = {}
    j, o = q0 + e, off
    while j < q1:
        v = y[j]
        n1 = y[j + 1] if j + 1 < C else 0
        if o < U:
            out[o] = v
        if v == n1:
            d = y[j + 2] if j + 2 < C else 0
            occ = (d - 256 if d >= 128 else d) - 48
            extra = (U - o - 1) if occ < 0 else max(occ - 1, 0)
            for t in range(1, extra + 1):
                if o + t < U:
                    out[o + t] = v
            o += 1 + extra
            j += 3
        else:
            o += 1
            j += 1
    return out
