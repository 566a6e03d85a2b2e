#!/bin/bash
# Second half of a GPU round (after tools/gpu_round.sh): the per-kind SQ counters of the codec
# kernels (tools/gpu_sq_kinds.sh -> tools/sq_kinds_table.py), the drop-in's call rates and the
# unchanged server side by side (tools/e2e_compare.py).   usage: bash tools/gpu_round_extras.sh TAG
set -o pipefail
TAG=${1:-round}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host_extras.txt
fatal() { case $1 in 124|134|137|139) exit $1;; esac; }
timeout -k 10 300 python -u -m pytest $R/tests/test_e2e_server.py -m gpu -s -q --timeout 240 --timeout-method thread > $O/e2e_extras.log 2>&1
rc=$?; echo "e2e rc=$rc" >> $O/status_extras; fatal $rc
E2E_TRACE_KEEP=$O/traces timeout -k 10 300 python -u $R/tools/e2e_trace.py > $O/e2e_trace.json 2> $O/e2e_trace.err
rc=$?; echo "e2e_trace rc=$rc" >> $O/status_extras; fatal $rc
bash $R/tools/gpu_sq_kinds.sh ${TAG}_sq k64_zero k64_random k64_runs50 k64_runs90 dec64k cfg1
rc=$?; echo "sq rc=$rc" >> $O/status_extras; fatal $rc
for T in 1 8 16; do
  echo "U=4096 threads=$T" >> $O/callrate.txt
  timeout -k 10 60 $R/tools/callrate $T 4096 2 >> $O/callrate.txt 2>&1
  rc=$?; echo "callrate $T rc=$rc" >> $O/status_extras; fatal $rc
done
for T in 1 8; do
  echo "U=32768 threads=$T" >> $O/callrate.txt
  timeout -k 10 60 $R/tools/callrate $T 32768 2 >> $O/callrate.txt 2>&1
  rc=$?; echo "callrate32k $T rc=$rc" >> $O/status_extras; fatal $rc
done
timeout -k 10 200 python -u $R/tools/call_latency_probe.py 0.3 > $O/call_latency.json 2> $O/call_latency.err
rc=$?; echo "call_latency rc=$rc" >> $O/status_extras; fatal $rc
timeout -k 10 500 python -u $R/tools/e2e_compare.py --reps 3 > $O/e2e_compare.json 2> $O/e2e_compare.err
rc=$?; echo "e2e_compare rc=$rc" >> $O/status_extras; fatal $rc
bash $R/tools/gpu_sq2.sh ${TAG}_sq2 k64_runs50 k64_zero cfg1
rc=$?; echo "sq2 rc=$rc" >> $O/status_extras; fatal $rc
exit 0
