#!/bin/bash
# Round 5 (r5x): one-buffer segmented launches without the plan and map kernels (RLE_SEG_ONE): the
# segmented, parity and host-path tests, same-process A/B against the five launches (segone0) on
# single large files and the mixed batch, and the drop-in's per-call latency with each build.
#   usage: bash tools/gpu_r5x.sh TAG
set -o pipefail
TAG=${1:-r5x}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_segmented.py $R/tests/test_gpu_parity.py $R/tests/test_gpu_hostpath.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 400 python -u $R/tools/ab_events.py --seg --workloads one4m,one64m,mixed --reps 10 --rounds 7 > $O/ab.json 2> $O/ab.err
rc=$?; echo "ab rc=$rc" >> $O/status
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 200 python -u $R/tools/call_latency_probe.py 0.3 > $O/lat_product.json 2> $O/lat_product.err
rc=$?; echo "lat product rc=$rc" >> $O/status
case $rc in 0) ;; *) exit $rc;; esac
RLE_MI355X_LIB=$R/c-filestorage-server-and-client_amd/build/variants/librle_segone0.so timeout -k 10 200 python -u $R/tools/call_latency_probe.py 0.3 > $O/lat_segone0.json 2> $O/lat_segone0.err
rc=$?; echo "lat segone0 rc=$rc" >> $O/status
exit $rc
