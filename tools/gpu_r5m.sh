#!/bin/bash
# Round 5: the drop-in's single compress calls of 64 KiB - 1 MiB through the one-pass encode
# (default) against the segmented kernels (RLE_MI355X_ENC_STREAM_MAX=0), after the parity tests.
#   usage: bash tools/gpu_r5m.sh TAG
set -o pipefail
TAG=${1:-r5m}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_stream.py $R/tests/test_gpu_hostpath.py $R/tests/test_gpu_fileops.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status
case $rc in 0) ;; *) exit $rc;; esac
for cfg in "pass:" "seg:RLE_MI355X_ENC_STREAM_MAX=0"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 200 python -u $R/tools/call_latency_probe.py 0.3 > $O/lat_$name.json 2> $O/lat_$name.err
  rc=$?; echo "lat $name rc=$rc" >> $O/status
  case $rc in 0) ;; *) exit $rc;; esac
done
exit 0
