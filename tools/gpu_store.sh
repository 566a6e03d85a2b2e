#!/bin/bash
# configs[1] bench line under each encode / decode store-policy combination.  usage: bash tools/gpu_store.sh TAG
set -o pipefail
TAG=${1:-st}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O
for E in wt wb; do for D in wt wb; do
  RLE_MI355X_STORE_ENC=$E RLE_MI355X_STORE_DEC=$D timeout -k 10 300 python $R/bench.py --steps 100 --no-cpu --no-north-star > $O/bench_$E$D.json 2> $O/bench_$E$D.err
  rc=$?; echo "$E $D rc=$rc" >> $O/status; [ $rc -ne 0 ] && exit $rc
done; done
exit 0
