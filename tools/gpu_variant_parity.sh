#!/bin/bash
# A/B timing of build/variants/librle_*.so against the product library, then the GPU parity suite
# run against each variant (RLE_MI355X_LIB).   usage: bash tools/gpu_variant_parity.sh TAG [workloads...]
set -o pipefail
TAG=${1:-var}; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 bash $R/tools/ab.sh $TAG/ab "$@"
rc=$?; echo "ab rc=$rc" >> $O/status; [ $rc -ne 0 ] && exit $rc
for SO in $R/c-filestorage-server-and-client_amd/build/variants/librle_*.so; do
  V=$(basename $SO .so)
  RLE_MI355X_LIB=$SO timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_$V.log 2>&1
  rc=$?; echo "pytest $V rc=$rc" >> $O/status
  case $rc in 0|1) ;; *) exit $rc;; esac
done
exit 0
