#!/bin/bash
# SQ counters of the large-batch decode: one wave per buffer against the decode in rounds
# (RLE_MI355X_DEC_ROUND), per workload, one --pmc pass each (kernel-trace-free).
# usage: bash tools/gpu_round_pmc.sh TAG "0 4" workload...
set -o pipefail
TAG=${1:-rpmc}; WIDTHS=$2; shift 2
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for WL in "$@"; do
  for W in $WIDTHS; do
    RLE_MI355X_DEC_ROUND=$W timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_${WL}_w$W -o run -- python3 $R/tools/prof_driver.py --workload $WL --reps 3 > $O/pmc_${WL}_w$W.log 2>&1
    rc=$?; echo "pmc $WL w$W rc=$rc" >> $O/status; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
