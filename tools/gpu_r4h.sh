#!/bin/bash
# Round-4 bench check: the one-rank timed loop replayed from one HIP graph (bench.py, default) and
# issued eagerly (RLE_BENCH_GRAPH=0), its GPU test, and the kernel trace of the graph form.
# usage: bash tools/gpu_r4h.sh TAG
set -o pipefail
TAG=${1:-r4h}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
fatal() { case $1 in 124|134|137|139) exit $1;; esac; }
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_bench.py -m gpu -v -rA --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status; fatal $rc
timeout -k 10 400 python $R/bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc" >> $O/status; fatal $rc
RLE_BENCH_GRAPH=0 timeout -k 10 400 python $R/bench.py --no-cpu > $O/bench_eager.json 2> $O/bench_eager.err
rc=$?; echo "bench eager rc=$rc" >> $O/status; fatal $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 20 --no-cpu --no-concurrent > $O/prof.log 2>&1
rc=$?; echo "prof rc=$rc" >> $O/status; fatal $rc
exit 0
