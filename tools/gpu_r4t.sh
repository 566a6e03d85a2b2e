#!/bin/bash
# Round-4: the issue-order sort without a memset (RLE_DEC_ORDER_PARTS): parity of the large-batch
# decodes, then same-process A/B against the global-histogram form (variant parts0) and the kernel
# trace of bench.py's dec64k.   usage: bash tools/gpu_r4t.sh TAG
set -o pipefail
TAG=${1:-r4t}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_parity.py -m gpu -v -rA --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 600 python -u $R/tools/ab_events.py --workloads dec64k,k64_random --reps 20 --rounds 9 > $O/ab.json 2> $O/ab.err
rc=$?; echo "ab rc=$rc" >> $O/status
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 400 python $R/bench.py --no-cpu --no-concurrent > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc" >> $O/status
exit $rc
