#!/bin/bash
# configs[1] kernel traces: the mixed batch beside its one-kind halves (per-SIMD balance check).
# usage: bash tools/gpu_c4k.sh TAG
set -o pipefail
TAG=${1:-c4k}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for WL in cfg1 c4k_random c4k_zero; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$WL -o run -- python3 $R/tools/prof_driver.py --workload $WL --reps 10 > $O/kt_$WL.log 2>&1
  rc=$?; echo "kt $WL rc=$rc" >> $O/status; [ $rc -ne 0 ] && exit $rc
done
exit 0
