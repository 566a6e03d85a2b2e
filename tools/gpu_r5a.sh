#!/bin/bash
# Round 5, first pass: ablation builds of the one-wave decode on the run-heavy 64 KiB kinds (which
# part of a general tile costs what), then the default bench line of the unchanged tree.
#   usage: bash tools/gpu_r5a.sh TAG
set -o pipefail
TAG=${1:-r5a}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
timeout -k 10 500 python -u $R/tools/ab_events.py --workloads k64_runs50,k64_runs90,k64_random --reps 10 --rounds 5 > $O/ab.json 2> $O/ab.err
rc=$?; echo "ab rc=$rc" >> $O/status
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 400 python $R/bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc" >> $O/status
exit $rc
