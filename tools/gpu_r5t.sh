#!/bin/bash
# Round 5 (r5t): the issue order in one launch from chunk-local sorts (RLE_ORDER_LOCAL): the batch
# decode tests past one residency round, same-process A/B against the global counting sort
# (ordglobal: memset + two launches), then the bench line.
#   usage: bash tools/gpu_r5t.sh TAG
set -o pipefail
TAG=${1:-r5t}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_parity.py $R/tests/test_gpu_fastpath.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 500 python -u $R/tools/ab_events.py --workloads dec64k,k64_zero,k64_runs50,s4k_mix --reps 10 --rounds 7 > $O/ab.json 2> $O/ab.err
rc=$?; echo "ab rc=$rc" >> $O/status
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 400 python $R/bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc" >> $O/status
exit $rc
