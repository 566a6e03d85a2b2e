#!/bin/bash
# Round 5 (r5s): segment summaries that sum their lanes once per segment (RLE_SEG_SUMDEFER): the
# segmented and fast-path parity tests, same-process A/B against per-tile sums (defer0) on the
# 1 MiB rows and the mixed batch, then a kernel trace of the product alone (summary / write split).
#   usage: bash tools/gpu_r5s.sh TAG
set -o pipefail
TAG=${1:-r5s}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_segmented.py $R/tests/test_gpu_fastpath.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 500 python -u $R/tools/ab_events.py --seg --workloads m1_zero,m1_random,m1_runs50,mixed --reps 5 --rounds 5 > $O/ab.json 2> $O/ab.err
rc=$?; echo "ab rc=$rc" >> $O/status
case $rc in 0) ;; *) exit $rc;; esac
mkdir -p /tmp/variants_off && mv $R/c-filestorage-server-and-client_amd/build/variants/* /tmp/variants_off/
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt -- python3 $R/tools/ab_events.py --seg --workloads m1_random,m1_runs50 --reps 3 --rounds 2 > $O/kt.log 2>&1
rc=$?; echo "kt rc=$rc" >> $O/status
exit $rc
