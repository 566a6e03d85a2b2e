#!/bin/bash
# Round 5 (r5w): the host registration probe (tools/probes/host_register_probe.cpp), then
# same-process A/B of the segment length cap (RLE_SEG_TILES_MAX 16 against 32 / 64) on the 1 MiB rows,
# the mixed configs[2] batch and one 64 MiB file.
#   usage: bash tools/gpu_r5w.sh TAG
set -o pipefail
TAG=${1:-r5w}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
timeout -k 10 120 $R/build/host_register_probe > $O/register.txt 2>&1
rc=$?; echo "register rc=$rc" >> $O/status
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 600 python -u $R/tools/ab_events.py --seg --workloads m1_zero,m1_random,m1_runs50,mixed,one64m --reps 5 --rounds 5 > $O/ab.json 2> $O/ab.err
rc=$?; echo "ab rc=$rc" >> $O/status
exit $rc
