#!/bin/bash
# Round 5: zero-copy calls up to 128 KiB of input (default) against 80 KiB (the zc80 variant), after
# the host-path parity tests.   usage: bash tools/gpu_r5n.sh TAG
set -o pipefail
TAG=${1:-r5n}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_hostpath.py $R/tests/test_gpu_fileops.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status
case $rc in 0) ;; *) exit $rc;; esac
V=$R/c-filestorage-server-and-client_amd/build/variants/librle_zc80.so
for cfg in "zc128:" "zc80:RLE_MI355X_LIB=$V" "zc128b:" "zc80b:RLE_MI355X_LIB=$V"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 200 python -u $R/tools/call_latency_probe.py 0.3 > $O/lat_$name.json 2> $O/lat_$name.err
  rc=$?; echo "lat $name rc=$rc" >> $O/status
  case $rc in 0) ;; *) exit $rc;; esac
done
exit 0
