#!/bin/bash
# Round-4 GPU pass f: zero-copy mid-size calls on the segmented kernels (RLE_MI355X_ZC_SEG) against
# the one-wave walk, parity first.   usage: bash tools/gpu_r4f.sh TAG
set -o pipefail
TAG=${1:-r4f}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
fatal() { case $1 in 124|134|137|139) exit $1;; esac; }
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_hostpath.py -k polled -m gpu -q -rA --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status; fatal $rc
for U in 8192 16384 24576 40000; do
  for Z in 0 8192; do
    for T in 1 8; do
      echo "zcseg=$Z U=$U threads=$T" >> $O/callrate_zcseg.txt
      RLE_MI355X_ZC_SEG=$Z timeout -k 10 60 $R/tools/callrate $T $U 1 >> $O/callrate_zcseg.txt 2>&1
      rc=$?; echo "callrate $Z $U $T rc=$rc" >> $O/status; fatal $rc
    done
  done
done
exit 0
