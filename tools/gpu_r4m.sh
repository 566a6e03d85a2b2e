#!/bin/bash
# Round-4: the parity module with the phase-map scan-skip edge test.   usage: bash tools/gpu_r4m.sh TAG
set -o pipefail
TAG=${1:-r4m}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_parity.py -m gpu -v -rA --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status
exit $rc
