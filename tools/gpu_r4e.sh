#!/bin/bash
# Round-4 GPU pass e: raw per-call traces of the e2e batteries (tools/e2e_trace.py, kept under
# gpurun_out/TAG/traces) and the side-by-side timing again (after the poll's spin-then-yield).
# usage: bash tools/gpu_r4e.sh TAG
set -o pipefail
TAG=${1:-r4e}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
fatal() { case $1 in 124|134|137|139) exit $1;; esac; }
E2E_TRACE_KEEP=$O/traces timeout -k 10 200 python -u $R/tools/e2e_trace.py > $O/e2e_trace.json 2> $O/e2e_trace.err
rc=$?; echo "e2e_trace rc=$rc" >> $O/status; fatal $rc
timeout -k 10 400 python -u $R/tools/e2e_compare.py --reps 2 > $O/e2e_compare.json 2> $O/e2e_compare.err
rc=$?; echo "e2e_compare rc=$rc" >> $O/status; fatal $rc
exit 0
