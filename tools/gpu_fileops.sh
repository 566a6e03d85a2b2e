#!/bin/bash
# File-op GPU tests and the fused / batched host-path measurements.  usage: bash tools/gpu_fileops.sh TAG
set -o pipefail
TAG=${1:-fo}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_fileops.py $R/tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u $R/tools/hostpath_bench.py --only fileops --seconds 0.5 > $O/fileops.json 2> $O/fileops.err
rc=$?; echo "fileops rc=$rc" >> $O/status
exit $rc
