#!/bin/bash
# Scheduler-strategy A/B (build/variants) + stamp shares of the diagnostic build.
# usage: bash tools/gpu_sched_ab.sh TAG
set -o pipefail
TAG=${1:-sched}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
RLE_MI355X_LIB=$R/c-filestorage-server-and-client_amd/build/variants/librle_stamps.so timeout -k 10 300 python3 $R/tools/stamps.py k64_zero k64_random k64_runs50 k64_runs90 cfg1 enc:k64_random enc:k64_zero enc:cfg1 > $O/stamps.txt 2>&1
rc=$?; echo "stamps rc=$rc" >> $O/status; case $rc in 124|134|137|139) exit $rc;; esac
mv $R/c-filestorage-server-and-client_amd/build/variants/librle_stamps.so $O/ 2>/dev/null
timeout -k 10 900 bash $R/tools/ab.sh $TAG/ab dec64k cfg1 k64_random k64_zero
