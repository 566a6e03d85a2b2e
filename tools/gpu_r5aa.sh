#!/bin/bash
# Round 5 (r5aa): chunk-local issue order in chunks of 256 buffers (one per thread) against 1024
# (per4): parity tests past one residency round, same-process A/B on the large decode batches.
#   usage: bash tools/gpu_r5aa.sh TAG
set -o pipefail
TAG=${1:-r5aa}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 400 python -u $R/tools/ab_events.py --workloads dec64k,k64_zero,s4k_mix --reps 12 --rounds 7 > $O/ab.json 2> $O/ab.err
rc=$?; echo "ab rc=$rc" >> $O/status
exit $rc
