#!/bin/bash
# Round 5: the timed region's fixed cost at the driver's settings (--steps 20 --warmup 5): graph
# replay or eager issue (RLE_BENCH_GRAPH), with or without the two HIP events inside the timed
# region (RLE_BENCH_TIMED_EVENTS), alternating, three times each.   usage: bash tools/gpu_r5i.sh TAG
set -o pipefail
TAG=${1:-r5i}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
for i in 1 2 3; do
  for v in "g1e1:1:1" "g1e0:1:0" "g0e1:0:1" "g0e0:0:0"; do
    name=${v%%:*}; rest=${v#*:}; g=${rest%%:*}; e=${rest#*:}
    RLE_BENCH_GRAPH=$g RLE_BENCH_TIMED_EVENTS=$e timeout -k 10 300 python $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-concurrent --no-north-star > $O/b_${name}_$i.json 2> $O/b_${name}_$i.err
    rc=$?; echo "bench $name $i rc=$rc" >> $O/status
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
exit 0
