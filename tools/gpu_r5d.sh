#!/bin/bash
# Round 5: the whole GPU suite after the literal paths' offsets moved from DPP scans to ballots
# (RLE_DEC_MBCNT, RLE_ENC_MBCNT), then same-process A/B against the scans (mbc0) and against the
# uniform-tile test in the one-round kernel too (uniall), and the bench line.
#   usage: bash tools/gpu_r5d.sh TAG
set -o pipefail
TAG=${1:-r5d}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
timeout -k 10 900 python -u -m pytest $R/tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 400 python -u $R/tools/ab_events.py --workloads cfg1,c4k_random,k64_random,k64_zero,k64_runs50,dec64k --reps 12 --rounds 5 > $O/ab.json 2> $O/ab.err
rc=$?; echo "ab rc=$rc" >> $O/status
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 400 python $R/bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc" >> $O/status
exit $rc
