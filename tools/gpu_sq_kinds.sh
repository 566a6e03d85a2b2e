#!/bin/bash
# Kernel trace + one SQ-counter pass (VALU / LDS / conflicts / wait) of the codec per workload.
# usage: bash tools/gpu_sq_kinds.sh TAG workload...   (PD_EXTRA: more prof_driver.py options, e.g. --seg)
set -o pipefail
TAG=${1:-sqk}; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for WL in "$@"; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$WL -o run -- python3 $R/tools/prof_driver.py --workload $WL $PD_EXTRA --warm 20 --reps 20 --rounds 3 > $O/kt_$WL.log 2>&1
  rc=$?; echo "kt $WL rc=$rc" >> $O/status; [ $rc -ne 0 ] && exit $rc
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_$WL -o run -- python3 $R/tools/prof_driver.py --workload $WL $PD_EXTRA --reps 3 > $O/pmc_$WL.log 2>&1
  rc=$?; echo "pmc $WL rc=$rc" >> $O/status; [ $rc -ne 0 ] && exit $rc
done
exit 0
