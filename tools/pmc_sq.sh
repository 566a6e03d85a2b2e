#!/bin/bash
# SQ activity counters for one workload (two passes of <= 8 SQ counters each, kernel-trace only).
# usage: bash tools/pmc_sq.sh TAG WORKLOAD   ->  gpurun_out/TAG/p1, p2 (tools/pmc_summary.py)
TAG=${1:-sq}; WL=${2:-cfg1}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
while read -r CTRS; do
  [ -z "$CTRS" ] && continue
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d $O/p$i -o run -- python3 $R/tools/prof_driver.py --workload $WL --reps 3 > $O/p$i.log 2>&1
  rc=$?
  echo "pass $i [$CTRS] rc=$rc" >> $O/status
  [ $rc -ne 0 ] && exit $rc
done <<'LIST'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM
LIST
exit 0
