#!/bin/bash
# Quick GPU iteration: parity tests, bench (no CPU leg), kernel trace of the dec64k and cfg1
# codec launches.   usage: bash tools/gpu_iter.sh TAG
set -o pipefail
TAG=${1:-iter}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python $R/bench.py --no-cpu > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc" >> $O/status
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
for WL in dec64k cfg1; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$WL -o run -- python3 $R/tools/prof_driver.py --workload $WL --reps 5 > $O/kt_$WL.log 2>&1
  rc=$?; echo "kt $WL rc=$rc" >> $O/status
  [ $rc -ne 0 ] && exit $rc
done
exit 0
