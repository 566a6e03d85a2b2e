#!/bin/bash
# Round-4: the resident service's stream at the greatest priority.  The queue probe with the spinner
# at each priority and with dependent launch pairs on the normal streams; the host-path parity
# tests; call rates (launch vs service); the e2e side by side (its service column).
# usage: bash tools/gpu_r4n.sh TAG
set -o pipefail
TAG=${1:-r4n}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
fatal() { case $1 in 124|134|137|139) exit $1;; esac; }
timeout -k 10 120 $R/build/queue_probe > $O/queue_probe.txt 2>&1
rc=$?; echo "queue_probe rc=$rc" >> $O/status; fatal $rc
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_hostpath.py -m gpu -q -rA --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status; fatal $rc
for S in 0 1; do
  for T in 1 8 16; do
    echo "service=$S U=4096 threads=$T" >> $O/callrate.txt
    RLE_MI355X_SERVICE=$S timeout -k 10 60 $R/tools/callrate $T 4096 1 >> $O/callrate.txt 2>&1
    rc=$?; echo "callrate service=$S $T rc=$rc" >> $O/status; fatal $rc
  done
done
timeout -k 10 500 python -u $R/tools/e2e_compare.py --reps 2 > $O/e2e_compare.json 2> $O/e2e_compare.err
rc=$?; echo "e2e_compare rc=$rc" >> $O/status; fatal $rc
E2E_TRACE_KEEP=$O/traces timeout -k 10 300 python -u $R/tools/e2e_trace.py > $O/e2e_trace.json 2> $O/e2e_trace.err
rc=$?; echo "e2e_trace rc=$rc" >> $O/status; fatal $rc
exit 0
