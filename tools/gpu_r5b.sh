#!/bin/bash
# Round 5: parity of the decode changes (fast-path and parity modules), the cost of the decode
# tile's analysis pieces (digit validation, uniform test, the literal path's attempt on run-heavy
# tiles) and of the single-value staging elision (RLE_DEC_VRUN) by same-process A/B, the segmented
# path issued as sub-batches (tools/seg_subbatch_probe.py), and the box's HBM write rate.
#   usage: bash tools/gpu_r5b.sh TAG
set -o pipefail
TAG=${1:-r5b}
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
timeout -k 10 400 python -u $R/tools/seg_subbatch_probe.py m1_random,m1_runs50,m1_zero > $O/subbatch.json 2> $O/subbatch.err
rc=$?; echo "subbatch rc=$rc" >> $O/status
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 120 python -u $R/tools/write_rate_probe.py > $O/write_rate.json 2> $O/write_rate.err
rc=$?; echo "write_rate rc=$rc" >> $O/status
exit $rc
