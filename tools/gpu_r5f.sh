#!/bin/bash
# Round 5: the cooperative kernels in rounds of 16 waves (encode up to 64 KiB, decode up to 80 tiles
# into 64 KiB; rle_coop_limits.h): their parity tests, then the drop-in's single calls with the
# zero-copy calls of 32-64 KiB in one workgroup (default) against the segmented form
# (RLE_MI355X_ZC_COOP=0), then the host-path test file.
#   usage: bash tools/gpu_r5f.sh TAG
set -o pipefail
TAG=${1:-r5f}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_coop.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_coop.log 2>&1
rc=$?; echo "pytest coop rc=$rc" >> $O/status
case $rc in 0) ;; *) exit $rc;; esac
for cfg in "coop:" "seg:RLE_MI355X_ZC_COOP=0"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 200 python -u $R/tools/call_latency_probe.py 0.3 > $O/lat_$name.json 2> $O/lat_$name.err
  rc=$?; echo "lat $name rc=$rc" >> $O/status
  case $rc in 0) ;; *) exit $rc;; esac
done
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_hostpath.py $R/tests/test_gpu_fileops.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_host.log 2>&1
rc=$?; echo "pytest host rc=$rc" >> $O/status
exit $rc
