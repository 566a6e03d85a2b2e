#!/bin/bash
# bench.py value against the timed step count (the driver runs
# --steps 20 --warmup 5): two runs of each configuration, fresh processes.
# usage: bash tools/bench_steps.sh TAG
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-bsteps}; mkdir -p $O
for rep in 1 2; do
  for cfg in "--steps 20 --warmup 5" "--steps 50" "--steps 200"; do
    timeout -k 10 300 python3 $R/bench.py --no-cpu --no-north-star $cfg > $O/run.json 2>/dev/null || exit $?
    python3 -c "
import json; d=json.loads(open('$O/run.json').read().strip().splitlines()[-1])
print('$cfg', '->', d['value'], 'GiB/s', d['ms_per_step'], 'ms/step')" >> $O/status
  done
done
cat $O/status
