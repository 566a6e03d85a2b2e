#!/bin/bash
# Round-4: the one-per-device service's call rate by thread count, its stream at the greatest and
# at the normal priority (RLE_MI355X_SERVICE_PRIO).   usage: bash tools/gpu_r4q.sh TAG
set -o pipefail
TAG=${1:-r4q}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
fatal() { case $1 in 124|134|137|139) exit $1;; esac; }
for P in 1 0; do
  for T in 1 2 4 8; do
    echo "prio_hi=$P threads=$T" >> $O/callrate.txt
    RLE_MI355X_SERVICE=1 RLE_MI355X_SERVICE_PRIO=$P timeout -k 10 60 $R/tools/callrate $T 4096 1 >> $O/callrate.txt 2>&1
    rc=$?; echo "callrate prio=$P $T rc=$rc" >> $O/status; fatal $rc
  done
done
exit 0
