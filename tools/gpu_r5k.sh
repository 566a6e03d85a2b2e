#!/bin/bash
# Round 5: the one-pass encode (a workgroup per buffer in rounds): its parity tests, then the timing
# probe against the segmented and one-wave encodes.   usage: bash tools/gpu_r5k.sh TAG
set -o pipefail
TAG=${1:-r5k}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_stream.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 400 python -u $R/tools/stream_probe.py m1_zero,m1_random,m1_runs50,k64_random,k64_runs50 > $O/stream.json 2> $O/stream.err
rc=$?; echo "probe rc=$rc" >> $O/status
exit $rc
