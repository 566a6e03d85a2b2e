#!/bin/bash
# One-wave-per-buffer vs segmented kernels on the same workloads (kernel trace of each).
# usage: bash tools/seg_compare.sh TAG [workloads...]
set -o pipefail
TAG=${1:-segcmp}; shift
WLS=${@:-mixed one4m one64m dec64k cfg1}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for WL in $WLS; do
  for MODE in one seg; do
    F=""; [ $MODE = seg ] && F="--seg"
    timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/${MODE}_$WL -o run -- python3 $R/tools/prof_driver.py --workload $WL --reps 5 $F > $O/${MODE}_$WL.log 2>&1
    rc=$?; echo "$MODE $WL rc=$rc $(tail -1 $O/${MODE}_$WL.log)" >> $O/status
    case $rc in 0|1) ;; *) exit $rc;; esac
  done
done
