#!/bin/bash
# Two PMC passes of SQ issue counters on one workload.  usage: bash tools/gpu_pmc2.sh TAG WORKLOAD [LIB]
set -o pipefail
TAG=${1:-pmc2}; WL=${2:-k64_random}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O
[ -n "$3" ] && export RLE_MI355X_LIB=$3
cd /tmp && export TMPDIR=/tmp
i=0
while read -r CTRS; do
  [ -z "$CTRS" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $CTRS --output-format csv -d $O/p$i -o run -- python3 $R/tools/prof_driver.py --workload $WL --reps 3 > $O/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc" >> $O/status; [ $rc -ne 0 ] && exit $rc
done <<'LIST'
SQ_CYCLES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INST_CYCLES_SALU SQ_INSTS SQ_IFETCH SQ_LDS_DATA_FIFO_FULL
SQ_LDS_CMD_FIFO_FULL SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU
GRBM_GUI_ACTIVE GRBM_COUNT
LIST
exit 0
