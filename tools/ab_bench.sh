#!/bin/bash
# A/B with bench.py's own timing (HIP events over 50 back-to-back launches per kernel): for the
# product library and each build/variants/librle_*.so, REPS alternating runs of
#   python bench.py --no-cpu --steps 50 [--workload W]
# and one line per run: library, workload, encode us, decode us, value.
# usage: bash tools/ab_bench.sh TAG [workload] [reps]
set -o pipefail
TAG=${1:-abb}; WL=${2:-cfg1}; REPS=${3:-3}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
for i in $(seq 1 $REPS); do
  for SO in $R/c-filestorage-server-and-client_amd/librle_mi355x.so $R/c-filestorage-server-and-client_amd/build/variants/librle_*.so; do
    V=$(basename $SO .so)
    RLE_MI355X_LIB=$SO timeout -k 10 300 python3 $R/bench.py --no-cpu --steps 50 --workload $WL > $O/${V}_${WL}_$i.json 2> $O/${V}_${WL}_$i.err
    rc=$?
    case $rc in 124|134|137|139) echo "$V rc=$rc" >> $O/status; exit $rc;; esac
    python3 -c "
import json,sys; d=json.loads(open('$O/${V}_${WL}_$i.json').read().strip().splitlines()[-1])
k=d['kernels']; print('$V', '$WL', 'enc %.2f dec %.2f value %.1f' % (k['encode']['us'], k['decode']['us'], d['value']))" >> $O/status
  done
done
cat $O/status
