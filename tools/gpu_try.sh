#!/bin/bash
# (tools/gpu_try.sh: used from the repo root as bash tools/gpu_try.sh ...)
# retry a gpurun call only while the pool has no free box (exit 3: nothing ran, nothing charged)
# usage: gpu_try.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 15); do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $LOG 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  grep -q "no free box\|backing off\|busy\|while being prepared" $LOG || exit $rc
  sleep 150
done
exit 3
