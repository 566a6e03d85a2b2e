#!/bin/bash
# Round-4: the north-star decode with and without the issue-order sort of large decode batches
# (RLE_MI355X_DEC_ORDER=0), bench.py's own dec64k measurement, fresh processes, interleaved twice.
# usage: bash tools/gpu_r4l.sh TAG
set -o pipefail
TAG=${1:-r4l}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
for i in 1 2; do
  for M in 1 0; do
    RLE_MI355X_DEC_ORDER=$M timeout -k 10 300 python $R/bench.py --no-cpu --no-concurrent > $O/bench_order${M}_$i.json 2> $O/bench_order${M}_$i.err
    rc=$?; echo "bench order=$M run $i rc=$rc" >> $O/status
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
exit 0
