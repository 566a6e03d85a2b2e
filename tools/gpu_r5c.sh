#!/bin/bash
# Round 5: parity with the uniform-tile test off (RLE_DEC_UNIFORM=0), same-process A/B of that
# change and of deeper tile rings for the large-batch decode (RLE_DEC_DEPTH_LARGE 3 / 4; 3 with
# 80-chunk staging), then the default bench line.   usage: bash tools/gpu_r5c.sh TAG
set -o pipefail
TAG=${1:-r5c}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
timeout -k 10 500 python -u -m pytest $R/tests/test_gpu_fastpath.py $R/tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 400 python -u $R/tools/ab_events.py --workloads k64_runs50,k64_runs90,k64_random,k64_zero,dec64k,cfg1 --reps 10 --rounds 5 > $O/ab.json 2> $O/ab.err
rc=$?; echo "ab rc=$rc" >> $O/status
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 400 python $R/bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc" >> $O/status
exit $rc
