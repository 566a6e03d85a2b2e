#!/bin/bash
# Round 5 (r5r): two literal tiles per step in the one-round decode kernel (dec_pair): the GPU suite,
# then same-process A/B against one tile per step (pair0) on configs[1], its two kinds and lone
# waves; the access-pattern probe (tools/probes/stream_pattern_probe.hip).
#   usage: bash tools/gpu_r5r.sh TAG
set -o pipefail
TAG=${1:-r5r}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
timeout -k 10 120 $R/build/stream_pattern_probe > $O/probe.txt 2>&1
rc=$?; echo "probe rc=$rc" >> $O/status
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 900 python -u -m pytest $R/tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 400 python -u $R/tools/ab_events.py --workloads cfg1,c4k_random,c4k_zero --reps 20 --rounds 9 > $O/ab.json 2> $O/ab.err
rc=$?; echo "ab rc=$rc" >> $O/status
case $rc in 0) ;; *) exit $rc;; esac
RLE_MI355X_COOP=0 timeout -k 10 300 python -u $R/tools/ab_events.py --workloads c4k_random_q --reps 20 --rounds 9 > $O/ab_q.json 2> $O/ab_q.err
rc=$?; echo "ab_q rc=$rc" >> $O/status
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 400 python $R/bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc" >> $O/status
exit $rc
