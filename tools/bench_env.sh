#!/bin/bash
# bench.py value (configs[1], --steps 50) under each environment setting of the product library,
# fresh processes, interleaved over 3 repetitions.   usage: bash tools/bench_env.sh TAG "ENV1 ENV2 ..."
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-benv}; ENVS=$2; mkdir -p $O
for rep in 1 2 3; do
  for E in $ENVS; do
    if [ "$E" = "-" ]; then
      timeout -k 10 300 python3 $R/bench.py --no-cpu --no-north-star --steps 50 > $O/run.json 2>>$O/err.log || exit $?
    else
      env "$E" timeout -k 10 300 python3 $R/bench.py --no-cpu --no-north-star --steps 50 > $O/run.json 2>>$O/err.log || exit $?
    fi
    python3 -c "
import json; d=json.loads(open('$O/run.json').read().strip().splitlines()[-1])
print('$E', '->', d['value'], 'GiB/s', d['ms_per_step'], 'ms/step', 'enc %.2f dec %.2f us' % (d['kernels']['encode']['us'], d['kernels']['decode']['us']))" >> $O/status
  done
done
cat $O/status
