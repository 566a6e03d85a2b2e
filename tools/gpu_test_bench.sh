#!/bin/bash
# GPU round: parity tests, then the bench, then a kernel-trace profile of the bench.
# usage: bash tools/gpu_test_bench.sh TAG [bench args...]
set -o pipefail
TAG=${1:-run}; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -m pytest $R/tests -m gpu -x -q > $O/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" | tee -a $O/status
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 400 python $R/bench.py "$@" > $O/bench.json 2> $O/bench.err || { echo "bench failed" | tee -a $O/status; exit 3; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 20 --no-cpu --no-concurrent > $O/prof.log 2>&1
echo "prof rc=$?" | tee -a $O/status
