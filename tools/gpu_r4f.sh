#!/bin/bash
# Round-4 GPU pass f: the per-context resident service and zero-copy mid-size calls on the
# segmented kernels (RLE_MI355X_ZC_SEG): parity first, then call rates by size and thread count.
# usage: bash tools/gpu_r4f.sh TAG
set -o pipefail
TAG=${1:-r4f}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
fatal() { case $1 in 124|134|137|139) exit $1;; esac; }
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_hostpath.py -k "polled or service" -m gpu -q -rA --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status; fatal $rc
for S in 0 1; do
  for T in 1 8 16; do
    echo "service=$S U=4096 threads=$T" >> $O/callrate_service.txt
    RLE_MI355X_SERVICE=$S timeout -k 10 60 $R/tools/callrate $T 4096 1 >> $O/callrate_service.txt 2>&1
    rc=$?; echo "callrate service=$S $T rc=$rc" >> $O/status; fatal $rc
  done
done
for U in 8192 16384 24576 40000; do
  for Z in 0 8192; do
    for T in 1 8; do
      echo "zcseg=$Z U=$U threads=$T" >> $O/callrate_zcseg.txt
      RLE_MI355X_ZC_SEG=$Z timeout -k 10 60 $R/tools/callrate $T $U 1 >> $O/callrate_zcseg.txt 2>&1
      rc=$?; echo "callrate $Z $U $T rc=$rc" >> $O/status; fatal $rc
    done
  done
done
E2E_TRACE_KEEP=$O/traces timeout -k 10 300 python -u $R/tools/e2e_trace.py > $O/e2e_trace.json 2> $O/e2e_trace.err
rc=$?; echo "e2e_trace rc=$rc" >> $O/status; fatal $rc
timeout -k 10 500 python -u $R/tools/e2e_compare.py --reps 2 > $O/e2e_compare.json 2> $O/e2e_compare.err
rc=$?; echo "e2e_compare rc=$rc" >> $O/status; fatal $rc
exit 0
