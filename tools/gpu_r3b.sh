#!/bin/bash
# r3b: exchange scan rewrite + async exchange: dist tests, scan timing under rocprof, bench in the
# three exchange modes at one rank, copy kernel nt A/B.
set -o pipefail
TAG=${1:-r3b}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc" >> $O/status; case $rc in 124|134|137|139) exit $rc;; esac; }
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_dist.py -m gpu -x -v -rA --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
chk $? pytest
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_scan -o run -- python3 $R/tools/dist_scan_prof.py > $O/scan.log 2>&1
chk $? prof_scan
cd $R
for M in async inline graph; do
  RLE_BENCH_FORCE_EXCHANGE=1 RLE_BENCH_XMODE=$M timeout -k 10 200 python $R/bench.py --steps 50 --warmup 5 --no-cpu --no-north-star --no-concurrent > $O/bench_x_$M.json 2> $O/bench_x_$M.err
  chk $? bench_x_$M
done
RLE_MI355X_COPY_NT=1 timeout -k 10 300 python $R/bench.py --steps 20 --warmup 5 --no-cpu --no-concurrent > $O/bench_nt.json 2> $O/bench_nt.err
chk $? bench_nt
