"""CPU pin of the algebra behind the fused append (RLEappend, include/rle_fileops.h),
checked with the oracle: for encoder output y = encode(x),

    encode(x ‖ new) = y[0, C - t) ‖ encode(head ‖ new)[16 - r :]

where c^L is x's final run, r = (L - 1) % 9 + 1 the length of the reference encoder's last token of
it (src/rleCompression.c:22-39; t = 1 byte when r = 1, else 3), and head = 16 - r filler bytes
(c^1, c^2 alternating) followed by c^r -- exactly what rle_append_prepare_device builds on the GPU.
Also pins the final-token check RLEappend uses to accept a stream for the incremental path."""
import numpy as np

import rle_oracle as O


def final_run(x):
    c = x[-1]
    L = 1
    while L < len(x) and x[-1 - L] == c:
        L += 1
    return c, L


def head_for(c, r):
    return bytes((c ^ (2 if (i & 1) else 1)) if i < 16 - r else c for i in range(16))


def spliced(y, x, new):
    c, L = final_run(x)
    r = (L - 1) % 9 + 1
    t = 1 if r == 1 else 3
    # the check RLEappend applies before keeping y[0, C - t)
    if t == 1:
        assert y[-1] == c
    else:
        assert y[-3] == c and y[-2] == c and y[-1] == ord("0") + r
    return y[:len(y) - t] + O.encode(head_for(c, r) + new)[16 - r:]


def test_filler_encodes_to_itself():
    for c in range(256):
        for r in range(1, 10):
            h = head_for(c, r)
            assert O.encode(h[:16 - r]) == h[:16 - r]
            assert h[15 - r] != c


def test_splice_identity_on_run_lengths():
    for ch in b"a9\x001":
        for L in range(1, 50):
            x = b"zq" + bytes([ch]) * L
            for new in (b"", bytes([ch]), bytes([ch]) * 17, b"k", bytes([ch]) * 3 + b"77"):
                assert spliced(O.encode(x), x, new) == O.encode(x + new), (ch, L, new)


def test_splice_identity_random():
    rng = np.random.default_rng(1)
    for i in range(2000):
        alpha = np.frombuffer([b"ab", b"9", b"123456789", bytes(range(256))][i % 4], np.uint8)
        n = int(rng.integers(1, 80))
        x = np.repeat(rng.choice(alpha, n), rng.integers(1, 25, n)).tobytes()
        m = int(rng.integers(0, 40))
        new = np.repeat(rng.choice(alpha, m), rng.integers(1, 25, m)).tobytes() if m else b""
        assert spliced(O.encode(x), x, new) == O.encode(x + new), (x, new)
