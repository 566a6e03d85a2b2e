#!/bin/bash
# Round-4 third GPU pass: small-call latency forms (tools/probes/mailbox_probe.hip: a launch per call
# against a resident service kernel polling a mailbox), hardware-queue sharing by stream priority,
# the resident small-call service of the drop-in (parity, call rate, e2e), and the call rate against
# the number of hardware queues the HIP runtime gives the process (GPU_MAX_HW_QUEUES; default 4).
# usage: bash tools/gpu_r4c.sh TAG
set -o pipefail
TAG=${1:-r4c}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
fatal() { case $1 in 124|134|137|139) exit $1;; esac; }
timeout -k 10 60 $R/build/mailbox_probe > $O/mailbox_probe.txt 2>&1
rc=$?; echo "mailbox_probe rc=$rc" >> $O/status; fatal $rc
timeout -k 10 60 $R/build/queue_probe > $O/queue_probe.txt 2>&1
rc=$?; echo "queue_probe rc=$rc" >> $O/status; fatal $rc
GPU_MAX_HW_QUEUES=8 timeout -k 10 60 $R/build/queue_probe > $O/queue_probe_q8.txt 2>&1
rc=$?; echo "queue_probe q8 rc=$rc" >> $O/status; fatal $rc
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_hostpath.py $R/tests/test_gpu_coop.py -m gpu -q -rA --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status; fatal $rc
for S in 0 1; do
  for T in 1 8 16; do
    echo "service=$S threads=$T" >> $O/callrate.txt
    RLE_MI355X_SERVICE=$S timeout -k 10 60 $R/tools/callrate $T 4096 2 >> $O/callrate.txt 2>&1
    rc=$?; echo "callrate service=$S $T rc=$rc" >> $O/status; fatal $rc
  done
done
for Q in 8 16; do
  echo "hwq=$Q threads=8" >> $O/callrate_hwq.txt
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 60 $R/tools/callrate 8 4096 2 >> $O/callrate_hwq.txt 2>&1
  rc=$?; echo "callrate hwq=$Q rc=$rc" >> $O/status; fatal $rc
done
timeout -k 10 400 python -u $R/tools/e2e_compare.py --reps 1 > $O/e2e_compare.json 2> $O/e2e_compare.err
rc=$?; echo "e2e_compare rc=$rc" >> $O/status; fatal $rc
exit 0
