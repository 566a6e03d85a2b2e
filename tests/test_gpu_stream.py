"""GPU parity of the one-pass encode (csrc/rle_coop.hip enc_stream_body: one workgroup per buffer
walking it in rounds of 4, 8 or 16 one-wave tiles, each input byte read once, a round's output
stored as it completes and its partial 16-byte chunk carried to the next round) against the oracle
and the compiled reference's golden vectors; bit-exact, output slots poisoned (nothing written past
C).  Measured no faster than the segmented encode (profiles/r5k_stream.md), so it
lives in the RLE_VARIANTS test library only: the checks run in a fresh process on that library."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PKG = os.path.join(ROOT, "c-filestorage-server-and-client_amd")
TESTLIB = os.path.join(PKG, "build", "librle_mi355x_testhooks.so")

_CODE = r'''
import sys
sys.path[:0] = sys.argv[1:4]
import numpy as np
import rle_mi355x as R
import rle_oracle as O
import json, os
from conftest import GOLDEN
from test_gpu_parity import gpu_encode
waves = int(sys.argv[4])
R.set_stream_waves(waves)

def check(xs, flags=0):
    ys, st = gpu_encode(xs, one_pass=True, flags=flags)
    assert (st == 0).all(), st
    bad = [i for i, x in enumerate(xs) if ys[i] != O.encode(x)]
    assert not bad, (len(bad), bad[:3], [len(xs[i]) for i in bad[:3]])

r = 1024 * waves   # one round's input
for kind in range(5):   # every kind at the round edges
    sizes = [0, 1, 2, 15, 16, 17, 1023, 1024, 1025, r - 1, r, r + 1, 2 * r - 16, 2 * r, 2 * r + 15, 3 * r + 7,
             65536, 100000, 262144 + 5]
    check([O.gen(kind, 17 * kind + i, s) for i, s in enumerate(sizes)])
check([O.gen(k, 900 + k, 1 << 20) for k in range(5)] + [O.gen(1, 7, (1 << 20) + 13)])
# runs and 3-byte tokens that end at, cross or start at a round edge, and the carried partial chunk
xs = []
for rl in range(1, 20):
    for side in (-1, 0, 1):
        x = bytearray(O.gen(1, 31 * rl + side, 3 * r + 40))
        for e in (r, 2 * r):
            lo = e - rl if side <= 0 else e
            hi = e + rl if side >= 0 else e
            x[lo:hi] = (b"7" if rl % 2 else b"\0") * (hi - lo)
        xs.append(bytes(x))
rng = np.random.default_rng(23)
for _ in range(64):
    s = int(rng.integers(1, 5 * r))
    alpha = np.frombuffer(rng.choice([b"a0123456789", b"\0\x01", b"33", b"ab", b"99"]), np.uint8)
    xs.append(np.repeat(rng.choice(alpha, size=s), rng.integers(1, 22, size=s))[:s].tobytes())
check(xs)
vec = json.load(open(os.path.join(GOLDEN, 'vectors.json')))
cases = [v for g in ("kat", "edge", "ladder", "fuzz") for v in vec[g]]
ys, st = gpu_encode([bytes.fromhex(v["in"]) for v in cases], one_pass=True)
assert ys == [bytes.fromhex(v["out"]) for v in cases] and (st == 0).all()
check([O.gen(k % 5, 40 + k, s) for k, s in enumerate([0, 5, 4096, 17000, 70000, 300001])],
      flags=R.RLE_LAUNCH_STATUS_FLAG)
print("ok")
'''


@pytest.mark.parametrize("waves", [16, 8, 4])
def test_one_pass_encode(waves):
    assert os.path.exists(TESTLIB), "build() makes the test library"
    env = dict(os.environ, RLE_MI355X_LIB=TESTLIB)
    r = subprocess.run([sys.executable, "-c", _CODE, PKG, os.path.join(ROOT, "oracle"), HERE, str(waves)], env=env,
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "ok" in r.stdout, (r.stdout[-1500:], r.stderr[-3000:])
