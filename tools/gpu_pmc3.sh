#!/bin/bash
# SQ issue / LDS counters (two passes) for one workload, product library and variants.
# usage: bash tools/gpu_pmc3.sh TAG WORKLOAD [variant .so ...]
set -o pipefail
TAG=${1:-pmc3}; WL=${2:-k64_random}; shift 2
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for SO in $R/c-filestorage-server-and-client_amd/librle_mi355x.so "$@"; do
  V=$(basename $SO .so)
  i=0
  while read -r CTRS; do
    [ -z "$CTRS" ] && continue
    i=$((i+1))
    RLE_MI355X_LIB=$SO timeout -k 10 240 rocprofv3 --pmc $CTRS --output-format csv -d $O/$V/p$i -o run -- python3 $R/tools/prof_driver.py --workload $WL --reps 3 > $O/$V.p$i.log 2>&1
    rc=$?; echo "$V pass $i rc=$rc" >> $O/status; case $rc in 124|134|137|139) exit $rc;; esac
  done <<'LIST'
SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_ACTIVE_INST_VALU2
SQ_CYCLES SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS SQ_IFETCH SQ_INSTS_BRANCH GRBM_GUI_ACTIVE
LIST
done
exit 0
