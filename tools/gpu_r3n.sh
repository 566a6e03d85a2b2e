#!/bin/bash
# r3n: per-wave timelines and the occupancy sweep with one wave per buffer (the cooperative kernels
# off), then the non-temporal hint and reversed segment order A/B.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3n
mkdir -p $O
for n in 256 1024 4096; do
  RLE_MI355X_COOP=0 RLE_MI355X_LIB=$GRAFT_REPO_ROOT/c-filestorage-server-and-client_amd/build/librle_tl.so timeout -k 10 120 python tools/timeline.py --workload c4k_random --n $n > $O/tl_$n.txt 2>&1 || exit $?
done
timeout -k 10 200 python tools/occupancy_sweep.py > $O/occ.json 2> $O/occ.err || exit $?
timeout -k 10 400 python tools/ab_events.py --workloads dec64k,k64_random,k64_zero,k64_runs50,k64_runs90,cfg1 --reps 5 --rounds 5 > $O/ab.json 2> $O/ab.err || exit $?
timeout -k 10 400 python tools/ab_events.py --seg --workloads m1_zero,m1_random,m1_runs50 --reps 5 --rounds 5 > $O/ab_seg.json 2> $O/ab_seg.err
