#!/bin/bash
# Round 5 (r5z): codec kernels instantiated per store policy (RLE_WT_STATIC: no run-time branch per
# store): parity and fast-path tests, same-process A/B against the run-time flag (wtdyn) on
# configs[1], its kinds and the 64 KiB batches.
#   usage: bash tools/gpu_r5z.sh TAG
set -o pipefail
TAG=${1:-r5z}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_parity.py $R/tests/test_gpu_fastpath.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 500 python -u $R/tools/ab_events.py --workloads cfg1,c4k_random,c4k_zero,dec64k,k64_runs50,k64_random --reps 12 --rounds 7 > $O/ab.json 2> $O/ab.err
rc=$?; echo "ab rc=$rc" >> $O/status
exit $rc
