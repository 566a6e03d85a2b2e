#!/bin/bash
# Round-4: the small-call rate against the hardware queues the HIP runtime gives the process
# (GPU_MAX_HW_QUEUES; default 4) and the configs[1] encode store policy (write-through, the default
# for batches of <= 4096 buffers, against write-back: kernel time and HBM write bytes).
# usage: bash tools/gpu_r4i.sh TAG
set -o pipefail
TAG=${1:-r4i}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
fatal() { case $1 in 124|134|137|139) exit $1;; esac; }
for Q in 4 8 16; do
  for T in 1 8 16; do
    echo "hwq=$Q threads=$T" >> $O/callrate_hwq.txt
    GPU_MAX_HW_QUEUES=$Q timeout -k 10 60 $R/tools/callrate $T 4096 2 >> $O/callrate_hwq.txt 2>&1
    rc=$?; echo "callrate hwq=$Q $T rc=$rc" >> $O/status; fatal $rc
  done
done
cd /tmp && export TMPDIR=/tmp
for P in wt wb; do
  RLE_MI355X_STORE_ENC=$P timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/kt_enc_$P -o run -- python3 $R/tools/prof_driver.py --workload cfg1 --reps 20 > $O/kt_enc_$P.log 2>&1
  rc=$?; echo "kt enc $P rc=$rc" >> $O/status; fatal $rc
  RLE_MI355X_STORE_ENC=$P timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_enc_$P -o run -- python3 $R/tools/prof_driver.py --workload cfg1 --reps 3 > $O/pmc_enc_$P.log 2>&1
  rc=$?; echo "pmc enc $P rc=$rc" >> $O/status; fatal $rc
done
exit 0
