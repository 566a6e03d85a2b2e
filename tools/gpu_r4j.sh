#!/bin/bash
# Round-4 parameter sweep of the one-wave kernels, same process (tools/ab_events.py): decode staging
# of large batches (RLE_DEC_CHUNKS_LARGE 128 / 192 against 96), decode waves per workgroup (1, 2
# against 4), decode wave priority (0, 2 against 1), encode waves per workgroup (2, 8 against 4),
# each against a `base` build of the same flags and the product library; parity of the product first.
# usage: bash tools/gpu_r4j.sh TAG
set -o pipefail
TAG=${1:-r4j}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_parity.py $R/tests/test_gpu_segmented.py $R/tests/test_gpu_coop.py -m gpu -q -rA --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 600 python -u $R/tools/ab_events.py --workloads cfg1,dec64k,k64_runs50,k64_runs90,k64_random,k64_zero --reps 20 --rounds 7 > $O/ab.json 2> $O/ab.err
rc=$?; echo "ab rc=$rc" >> $O/status
exit $rc
