#!/bin/bash
# Round-4 GPU pass d: the fixed exchange / coalescing tests, small-call cost by size for the
# zero-copy and the copying forms (RLE_MI355X_SMALL), and the segmented uniform-tile A/B repeated.
# usage: bash tools/gpu_r4d.sh TAG
set -o pipefail
TAG=${1:-r4d}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
fatal() { case $1 in 124|134|137|139) exit $1;; esac; }
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_dist.py $R/tests/test_gpu_hostpath.py -m gpu -q -rA --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status; fatal $rc
for U in 4096 8192 16384 40000; do
  for M in zc copy; do
    for T in 1 8; do
      echo "small=$M U=$U threads=$T" >> $O/callrate_size.txt
      if [ $M = copy ]; then export RLE_MI355X_SMALL=copy; else unset RLE_MI355X_SMALL; fi
      timeout -k 10 60 $R/tools/callrate $T $U 1 >> $O/callrate_size.txt 2>&1
      rc=$?; echo "callrate $M $U $T rc=$rc" >> $O/status; fatal $rc
    done
  done
done
unset RLE_MI355X_SMALL
timeout -k 10 300 python -u $R/tools/ab_events.py --seg --workloads mixed,m1_random,m1_runs50 --reps 5 --rounds 9 > $O/ab_seg.json 2> $O/ab_seg.err
rc=$?; echo "ab_seg rc=$rc" >> $O/status; fatal $rc
exit 0
