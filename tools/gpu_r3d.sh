#!/bin/bash
# r3d: host path (staging modes, coalescing, e2e side by side), exchange scan, SQ counters per kind.
set -o pipefail
TAG=${1:-r3d}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc" >> $O/status; case $rc in 124|134|137|139) exit $rc;; esac; [ $rc -ne 0 ] && exit $rc; }
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_hostpath.py $R/tests/test_gpu_dist.py $R/tests/test_gpu_fileops.py $R/tests/test_e2e_server.py -m gpu -x -v -rA --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
chk $? pytest
for T in 1 2 4 8 16; do
  for C in 1 0; do
    RLE_MI355X_COALESCE=$C timeout -k 10 60 $R/tools/callrate $T 4096 2 >> $O/callrate.jsonl 2>> $O/callrate.err
    chk $? callrate_${T}_$C
  done
done
timeout -k 10 400 python $R/tools/e2e_compare.py --reps 3 > $O/e2e.json 2> $O/e2e.err
chk $? e2e
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_scan -o run -- python3 $R/tools/dist_scan_prof.py > $O/scan.log 2>&1
chk $? prof_scan
for WL in cfg1 k64_random k64_zero k64_runs50 k64_runs90; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$WL -o run -- python3 $R/tools/prof_driver.py --workload $WL --reps 5 > $O/kt_$WL.log 2>&1
  chk $? kt_$WL
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU --output-format csv -d $O/pmc_$WL -o run -- python3 $R/tools/prof_driver.py --workload $WL --reps 3 > $O/pmc_$WL.log 2>&1
  chk $? pmc_$WL
done
