#!/bin/bash
# r3p: two tiles per step (small-buffer encode, one-round decode): GPU parity, then A/B against one tile per step.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3p
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 400 python tools/ab_events.py --workloads cfg1,c4k_random,c4k_zero,c4k_runs50,s4k_mix,dec64k --reps 10 --rounds 7 > $O/ab.json 2> $O/ab.err
