#!/bin/bash
# The decode scatter writing token starts only (RLE_SCAT_MASK=1, variant build `scatmask`) against
# the product's per-position scatter: same-process A/B on the run-heavy 64 KiB batches, then one SQ
# counter pass (LDS bank conflicts, LDS and VALU instructions) per build and kind.
#   usage: bash tools/gpu_scatmask_pmc.sh [TAG]
set -o pipefail
TAG=${1:-r5ad}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 400 python -u $R/tools/ab_events.py --workloads k64_runs50,k64_runs90,dec64k --reps 8 --rounds 5 > $O/ab.json 2> $O/ab.err || exit $?
cd /tmp && export TMPDIR=/tmp
for V in product scatmask; do
  if [ $V = product ]; then unset RLE_MI355X_LIB; else export RLE_MI355X_LIB=$R/c-filestorage-server-and-client_amd/build/variants/librle_$V.so; fi
  for WL in k64_runs50 k64_runs90; do
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_${V}_$WL -o run -- python3 $R/tools/prof_driver.py --workload $WL --reps 3 > $O/pmc_${V}_$WL.log 2>&1 || exit $?
  done
done
exit 0
