#!/bin/bash
# Round 5 (r5y): the plan kernel writes the segments' buffers below 4096 buffers (RLE_PLAN_MAP, one
# launch fewer per segmented call): segmented and parity tests, same-process A/B against the
# separate map launch (planmap0) on the mixed configs[2] batch and the 1 MiB rows.
#   usage: bash tools/gpu_r5y.sh TAG
set -o pipefail
TAG=${1:-r5y}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_segmented.py $R/tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 400 python -u $R/tools/ab_events.py --seg --workloads mixed,m1_zero,m1_random --reps 10 --rounds 7 > $O/ab.json 2> $O/ab.err
rc=$?; echo "ab rc=$rc" >> $O/status
exit $rc
