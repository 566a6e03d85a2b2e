#!/bin/bash
# Round 5 (r5u): scalar-unit counters of the configs[1] kernels (is the one-round decode / encode
# bound by SALU issue?): the counter list of this box, then one SQ pass per workload.
#   usage: bash tools/gpu_r5u.sh TAG workload...
set -o pipefail
TAG=${1:-r5u}; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1
echo "list rc=$?" >> $O/status
for WL in "$@"; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_$WL -o run -- python3 $R/tools/prof_driver.py --workload $WL --reps 3 > $O/pmc_$WL.log 2>&1
  rc=$?; echo "pmc $WL rc=$rc" >> $O/status; [ $rc -ne 0 ] && exit $rc
done
exit 0
