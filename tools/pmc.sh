#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only, no sys/runtime traces).
# usage: bash tools/pmc.sh TAG WORKLOAD
TAG=${1:-pmc}; WL=${2:-dec64k}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
while read -r CTRS; do
  [ -z "$CTRS" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $CTRS --output-format csv -d $O/p$i -o run -- python3 $R/tools/prof_driver.py --workload $WL --reps 3 > $O/p$i.log 2>&1
  rc=$?
  echo "pass $i [$CTRS] rc=$rc" >> $O/status
  case $rc in 124|134|137|139) exit $rc;; esac
done <<'LIST'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE
FETCH_SIZE
WRITE_SIZE
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM
SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM
LIST
