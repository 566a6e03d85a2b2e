#!/bin/bash
# Per-kind kernel trace (+ one PMC pass of SQ counters) of the codec, steady state: 20 warm encodes
# and decodes, then 3 rounds of 20 each (tools/kinds_table.py --skip 21).
#   usage: bash tools/gpu_kinds.sh TAG [pmc]
set -o pipefail
TAG=${1:-kinds}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for WL in k64_zero k64_random k64_runs50 k64_runs90 dec64k cfg1; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$WL -o run -- python3 $R/tools/prof_driver.py --workload $WL --warm 20 --reps 20 --rounds 3 > $O/kt_$WL.log 2>&1
  rc=$?; echo "kt $WL rc=$rc" >> $O/status; [ $rc -ne 0 ] && exit $rc
done
if [ "$2" = "pmc" ]; then
  for WL in k64_zero k64_random; do
    timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/pmc_$WL/p1 -o run -- python3 $R/tools/prof_driver.py --workload $WL --reps 3 > $O/pmc_$WL.log 2>&1
    rc=$?; echo "pmc $WL rc=$rc" >> $O/status; [ $rc -ne 0 ] && exit $rc
  done
fi
exit 0
