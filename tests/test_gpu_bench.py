"""bench.py at one rank on the GPU (the driver's N = 1 run, shortened): the timed loop issues the K
steps eagerly (the default since round 6) or replays them from one HIP graph (RLE_BENCH_GRAPH=1), the
round trip is verified, the other issue form is timed beside it (value_eager and value_graph both
in the line, `value` the faster of them), and the per-kernel split of the timed loop's GPU time stays below the step time
(VERDICT r3 item 5)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("graph", ["1", "0"])
def test_bench_one_rank(graph):
    env = dict(os.environ, RLE_BENCH_GRAPH=graph)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "8", "--warmup", "3", "--no-cpu",
                        "--no-north-star", "--no-concurrent"], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["verified_bit_exact_roundtrip"] is True
    assert out["value"] == max(out["value_eager"], out["value_graph"]), out
    assert out["kernels"]["roundtrip"]["us"] <= out["ms_per_step"] * 1000 * 1.02, (out["kernels"], out["ms_per_step"])
    assert out["value_eager"] > 0 and out["value_graph"] > 0, out
    assert ("graph" in out["issue"].split("(")[0]) is (out["value_graph"] > out["value_eager"]), out["issue"]
