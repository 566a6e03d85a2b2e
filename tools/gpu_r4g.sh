#!/bin/bash
# Round-4 GPU pass g: the drop-in's small-call paths after r4f (resident service: one acquire and one
# release per request; start-up pool; zero-copy segmented default from 32 KiB): the host-path and
# coop parity tests, call rates (launch vs service, 1/8/16 threads; sizes), the e2e side by side and
# its traces.   usage: bash tools/gpu_r4g.sh TAG
set -o pipefail
TAG=${1:-r4g}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
fatal() { case $1 in 124|134|137|139) exit $1;; esac; }
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_hostpath.py $R/tests/test_gpu_coop.py $R/tests/test_gpu_fileops.py -m gpu -q -rA --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status; fatal $rc
for S in 0 1; do
  for T in 1 8 16; do
    echo "service=$S U=4096 threads=$T" >> $O/callrate.txt
    RLE_MI355X_SERVICE=$S timeout -k 10 60 $R/tools/callrate $T 4096 1 >> $O/callrate.txt 2>&1
    rc=$?; echo "callrate service=$S $T rc=$rc" >> $O/status; fatal $rc
  done
done
for U in 16384 40000 65536; do
  for S in 0 1; do
    echo "service=$S U=$U threads=1" >> $O/callrate.txt
    RLE_MI355X_SERVICE=$S timeout -k 10 60 $R/tools/callrate 1 $U 1 >> $O/callrate.txt 2>&1
    rc=$?; echo "callrate service=$S U=$U rc=$rc" >> $O/status; fatal $rc
  done
done
E2E_TRACE_KEEP=$O/traces timeout -k 10 300 python -u $R/tools/e2e_trace.py > $O/e2e_trace.json 2> $O/e2e_trace.err
rc=$?; echo "e2e_trace rc=$rc" >> $O/status; fatal $rc
timeout -k 10 500 python -u $R/tools/e2e_compare.py --reps 2 > $O/e2e_compare.json 2> $O/e2e_compare.err
rc=$?; echo "e2e_compare rc=$rc" >> $O/status; fatal $rc
exit 0
