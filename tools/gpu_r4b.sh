#!/bin/bash
# Round-4 second GPU pass: small-call probes (a launch per call against a resident mailbox service;
# hardware-queue sharing by stream priority), the -m gpu suite (e2e last), the decode A/Bs (uniform
# tiles), launch-timing modes, e2e side by side (incl. the resident service) and its per-call trace,
# and the call rate (polled launch, hipStreamSynchronize, resident service).
# usage: bash tools/gpu_r4b.sh TAG
set -o pipefail
TAG=${1:-r4b}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
fatal() { case $1 in 124|134|137|139) exit $1;; esac; }
timeout -k 10 60 $R/build/mailbox_probe > $O/mailbox_probe.txt 2>&1
rc=$?; echo "mailbox_probe rc=$rc" >> $O/status; fatal $rc
timeout -k 10 60 $R/build/queue_probe > $O/queue_probe.txt 2>&1
rc=$?; echo "queue_probe rc=$rc" >> $O/status; fatal $rc
timeout -k 10 700 python -u -m pytest $R/tests -m gpu -q -rA --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status; fatal $rc
timeout -k 10 300 python -u $R/tools/ab_events.py --workloads cfg1,dec64k,k64_zero,c4k_zero --reps 10 --rounds 5 > $O/ab.json 2> $O/ab.err
rc=$?; echo "ab rc=$rc" >> $O/status; fatal $rc
timeout -k 10 300 python -u $R/tools/ab_events.py --seg --workloads m1_zero,mixed --reps 5 --rounds 5 > $O/ab_seg.json 2> $O/ab_seg.err
rc=$?; echo "ab_seg rc=$rc" >> $O/status; fatal $rc
for S in 0 1; do
  for T in 1 8 16; do
    echo "service=$S threads=$T" >> $O/callrate.txt
    RLE_MI355X_SERVICE=$S timeout -k 10 60 $R/tools/callrate $T 4096 2 >> $O/callrate.txt 2>&1
    rc=$?; echo "callrate service=$S $T rc=$rc" >> $O/status; fatal $rc
  done
done
for T in 1 8; do
  echo "poll=0 threads=$T" >> $O/callrate.txt
  RLE_MI355X_POLL=0 timeout -k 10 60 $R/tools/callrate $T 4096 2 >> $O/callrate.txt 2>&1
  rc=$?; echo "callrate poll=0 $T rc=$rc" >> $O/status; fatal $rc
done
timeout -k 10 400 python -u $R/tools/e2e_compare.py --reps 2 > $O/e2e_compare.json 2> $O/e2e_compare.err
rc=$?; echo "e2e_compare rc=$rc" >> $O/status; fatal $rc
timeout -k 10 200 python -u $R/tools/e2e_trace.py > $O/e2e_trace.json 2> $O/e2e_trace.err
rc=$?; echo "e2e_trace rc=$rc" >> $O/status; fatal $rc
timeout -k 10 300 python -u $R/tools/launch_modes.py > $O/launch_modes.json 2> $O/launch_modes.err
rc=$?; echo "launch_modes rc=$rc" >> $O/status; fatal $rc
exit 0
