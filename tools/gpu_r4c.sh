#!/bin/bash
# Round-4 third GPU pass: small-call latency forms (tools/probes/mailbox_probe.hip: a launch per call
# against a resident service kernel polling a mailbox) and the call rate against the number of
# hardware queues the HIP runtime gives the process (GPU_MAX_HW_QUEUES; 4 is its default).
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
for Q in 4 8 16; do
  for T in 1 8 16; do
    echo "hwq=$Q threads=$T" >> $O/callrate_hwq.txt
    GPU_MAX_HW_QUEUES=$Q timeout -k 10 60 $R/tools/callrate $T 4096 2 >> $O/callrate_hwq.txt 2>&1
    rc=$?; echo "callrate hwq=$Q $T rc=$rc" >> $O/status; fatal $rc
  done
done
exit 0
