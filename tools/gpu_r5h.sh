#!/bin/bash
# Round 5: the bench line at the driver's own settings (--steps 20 --warmup 5) with the timed steps
# replayed from one HIP graph (RLE_BENCH_GRAPH=1, the round-4 default) and issued eagerly
# (RLE_BENCH_GRAPH=0), alternating, three times each; then once each at the defaults (50 / 10).
#   usage: bash tools/gpu_r5h.sh TAG
set -o pipefail
TAG=${1:-r5h}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
for i in 1 2 3; do
  for g in 1 0; do
    RLE_BENCH_GRAPH=$g timeout -k 10 300 python $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-concurrent --no-north-star > $O/bench_s20_g${g}_$i.json 2> $O/bench_s20_g${g}_$i.err
    rc=$?; echo "bench s20 g$g $i rc=$rc" >> $O/status
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
for g in 1 0; do
  RLE_BENCH_GRAPH=$g timeout -k 10 300 python $R/bench.py --no-cpu --no-concurrent --no-north-star > $O/bench_def_g$g.json 2> $O/bench_def_g$g.err
  rc=$?; echo "bench def g$g rc=$rc" >> $O/status
  case $rc in 0) ;; *) exit $rc;; esac
done
exit 0
