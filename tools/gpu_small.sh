#!/bin/bash
# Drop-in tests and single-call host-path rates with the small-call path copying (default) and
# zero-copy (RLE_MI355X_SMALL=zerocopy).   usage: bash tools/gpu_small.sh TAG
set -o pipefail
TAG=${1:-sm}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O
RLE_MI355X_SMALL=zerocopy timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_parity.py $R/tests/test_gpu_fileops.py -x -q --timeout 120 --timeout-method thread > $O/pytest_zc.log 2>&1
rc=$?; echo "pytest zc rc=$rc" >> $O/status; [ $rc -ne 0 ] && exit $rc
for M in copy zerocopy; do
  RLE_MI355X_SMALL=$M timeout -k 10 300 python -u $R/tools/hostpath_bench.py --only single --seconds 0.3 > $O/single_$M.json 2> $O/single_$M.err
  rc=$?; echo "single $M rc=$rc" >> $O/status; [ $rc -ne 0 ] && exit $rc
done
exit 0
