#!/bin/bash
# Second SQ-counter pass per workload: scalar / branch / LDS issue and waits beside the VALU pass of
# tools/gpu_sq_kinds.sh (where the run-heavy decode tiles spend their issue cycles).
# usage: bash tools/gpu_sq2.sh TAG workload...
set -o pipefail
TAG=${1:-sq2}; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for WL in "$@"; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/pmc2_$WL -o run -- python3 $R/tools/prof_driver.py --workload $WL --reps 3 > $O/pmc2_$WL.log 2>&1
  rc=$?; echo "pmc2 $WL rc=$rc" >> $O/status; [ $rc -ne 0 ] && exit $rc
done
exit 0
