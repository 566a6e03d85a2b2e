#!/bin/bash
# bench.py value at the driver's step count under each host wait mode (RLE_BENCH_SCHED), fresh
# processes, interleaved.   usage: bash tools/bench_sched.sh TAG
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-bsched}; mkdir -p $O
for rep in 1 2 3; do
  for m in auto spin yield; do
    RLE_BENCH_SCHED=$m timeout -k 10 300 python3 $R/bench.py --no-cpu --no-north-star --steps 20 --warmup 5 > $O/run.json 2>>$O/err.log || exit $?
    python3 -c "
import json; d=json.loads(open('$O/run.json').read().strip().splitlines()[-1])
print('$m', d.get('host_wait'), '->', d['value'], 'GiB/s', d['ms_per_step'], 'ms/step')" >> $O/status
  done
done
cat $O/status
