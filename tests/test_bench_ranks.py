"""CPU tests of bench.py's multi-rank path (`--gpus N` used to be ignored).

`bench.py --gpus N --dry-run` starts N rank processes itself (no WORLD_SIZE in the environment),
forms a gloo process group of N ranks over 127.0.0.1, and runs the same rank loop as on the GPUs --
shard layout, exchange (the torch fallback: all_gather_into_tensor + global-order scan), barriers,
max-over-ranks timing, rank-0 JSON line -- with the codec launches left out.  The exchange's
offsets are checked on every rank against a closed form of the global sizes."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout, env=env)


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_flag_spawns_ranks(n):
    r = _run(["--dry-run", "--gpus", str(n), "--steps", "3", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout   # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == n
    assert out["dry_run"] is True
    assert out["steps"] == 3 and out["warmup"] == 1
    assert out["exchange"]["mode"] == "torch"
    assert out["exchange"]["offsets_match_process_group"] is True
    assert out["config"]["buffers_per_gpu"] == 4096
    assert out["value"] > 0 and out["scaling"] == "weak"


def test_failed_rank_stops_the_others():
    # rank 1 exits before the rendezvous: rank 0 would wait in init_process_group forever; the
    # launcher must notice, stop it and return the failure
    r = _run(["--dry-run", "--gpus", "2", "--steps", "2", "--warmup", "1"], {"RLE_BENCH_DRY_FAIL_RANK": "1"},
             timeout=120)
    assert r.returncode == 3
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_single_rank_dry_run():
    r = _run(["--dry-run", "--steps", "2", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["n_gpus"] == 1 and "exchange" not in out
