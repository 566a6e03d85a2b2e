#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per codec launch (one counter per pass) for the given workloads.
# usage: bash tools/gpu_pmc_kinds.sh TAG workload...
set -o pipefail
TAG=${1:-pk}; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for WL in "$@"; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 240 rocprofv3 --pmc $C --output-format csv -d $O/pmc_${WL}_$C -o run -- python3 $R/tools/prof_driver.py --workload $WL --reps 3 > $O/pmc_${WL}_$C.log 2>&1
    rc=$?; echo "pmc $WL $C rc=$rc" >> $O/status
    case $rc in 124|134|137|139) exit $rc;; esac
  done
done
exit 0
