#!/bin/bash
# Parity suite (GPU tests only, stop at first failure) then per-kind traces (+PMC).  usage: bash tools/gpu_quick.sh TAG [pmc]
set -o pipefail
TAG=${1:-q}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status; [ $rc -ne 0 ] && exit $rc
bash $R/tools/gpu_kinds.sh $TAG $2
