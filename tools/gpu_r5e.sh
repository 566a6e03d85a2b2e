#!/bin/bash
# Round 5: the drop-in's single calls with the deep tile ring for few-buffer launches
# (RLE_FEW_DEPTH, product 8 against the few2 variant), with and without the zero-copy segmented
# form from 32 KiB (RLE_MI355X_ZC_SEG), after the host-path and parity tests.
#   usage: bash tools/gpu_r5e.sh TAG
set -o pipefail
TAG=${1:-r5e}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_hostpath.py $R/tests/test_gpu_parity.py $R/tests/test_gpu_fileops.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status
case $rc in 0) ;; *) exit $rc;; esac
V=$R/c-filestorage-server-and-client_amd/build/variants/librle_few2.so
for cfg in "prod:" "prod_zc0:RLE_MI355X_ZC_SEG=0" "few2:RLE_MI355X_LIB=$V" "few2_zc0:RLE_MI355X_LIB=$V RLE_MI355X_ZC_SEG=0"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 200 python -u $R/tools/call_latency_probe.py 0.3 > $O/lat_$name.json 2> $O/lat_$name.err
  rc=$?; echo "lat $name rc=$rc" >> $O/status
  case $rc in 0) ;; *) exit $rc;; esac
done
exit 0
