#!/bin/bash
# Drop-in GPU tests, then the host-path single-call rates under each staging mode (RLE_MI355X_STAGING).
# usage: bash tools/gpu_staging.sh TAG
set -o pipefail
TAG=${1:-stg}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_parity.py $R/tests/test_gpu_fileops.py $R/tests/test_gpu_segmented.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status; [ $rc -ne 0 ] && exit $rc
for M in pinned pipe direct; do
  RLE_MI355X_STAGING=$M timeout -k 10 300 python -u $R/tools/hostpath_bench.py --only single --seconds 0.3 > $O/single_$M.json 2> $O/single_$M.err
  rc=$?; echo "single $M rc=$rc" >> $O/status; [ $rc -ne 0 ] && exit $rc
done
exit 0
