#!/bin/bash
# Round-4 first GPU pass: the whole -m gpu suite on the new host-side code, the per-kind SQ
# counters, the e2e side-by-side and the call rate.   usage: bash tools/gpu_r4a.sh TAG
set -o pipefail
TAG=${1:-r4a}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
fatal() { case $1 in 124|134|137|139) exit $1;; esac; }
timeout -k 10 60 $R/build/sync_probe > $O/sync_probe.txt 2>&1
rc=$?; echo "sync_probe rc=$rc" >> $O/status; fatal $rc
timeout -k 10 60 $R/build/store_probe > $O/store_probe.txt 2>&1
rc=$?; echo "store_probe rc=$rc" >> $O/status; fatal $rc
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q -rA --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status; fatal $rc
timeout -k 10 300 python -u $R/tools/ab_events.py --workloads cfg1,dec64k,k64_runs50,k64_runs90,k64_random,k64_zero --reps 10 --rounds 5 > $O/ab.json 2> $O/ab.err
rc=$?; echo "ab rc=$rc" >> $O/status; fatal $rc
bash $R/tools/gpu_sq_kinds.sh ${TAG}_sq k64_zero k64_random k64_runs50 k64_runs90 cfg1
rc=$?; echo "sq rc=$rc" >> $O/status; fatal $rc
timeout -k 10 300 python -u $R/tools/e2e_compare.py --reps 2 > $O/e2e_compare.json 2> $O/e2e_compare.err
rc=$?; echo "e2e_compare rc=$rc" >> $O/status; fatal $rc
for T in 1 8 16; do
  timeout -k 10 60 $R/tools/callrate $T 4096 2 >> $O/callrate.txt 2>&1
  rc=$?; echo "callrate $T rc=$rc" >> $O/status; fatal $rc
done
exit 0
