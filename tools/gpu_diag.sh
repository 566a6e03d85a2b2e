#!/bin/bash
# Diagnostics: pattern ceilings (store/issue probes), per-kind decode/encode kernel trace,
# stamp shares of the diagnostic build.   usage: bash tools/gpu_diag.sh TAG
set -o pipefail
TAG=${1:-diag}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 120 $R/build/store_probe > $O/store_probe.txt 2>&1; echo "store rc=$?" >> $O/status
timeout -k 10 120 $R/build/issue_probe > $O/issue_probe.txt 2>&1; echo "issue rc=$?" >> $O/status
RLE_MI355X_LIB=$R/c-filestorage-server-and-client_amd/build/variants/librle_stamps.so timeout -k 10 300 python3 $R/tools/stamps.py k64_zero k64_random k64_runs50 k64_runs90 cfg1 enc:k64_random enc:k64_zero > $O/stamps.txt 2>&1
rc=$?; echo "stamps rc=$rc" >> $O/status; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
for WL in k64_zero k64_random k64_runs50 k64_runs90; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$WL -o run -- python3 $R/tools/prof_driver.py --workload $WL --reps 5 > $O/kt_$WL.log 2>&1
  rc=$?; echo "kt $WL rc=$rc" >> $O/status; [ $rc -ne 0 ] && exit $rc
done
exit 0
