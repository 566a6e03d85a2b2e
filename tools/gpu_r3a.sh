#!/bin/bash
# r3 first GPU pass: parity (incl. the new configs[3] full-shard and exchange tests), bench at N=1,
# the N>1 rank loop rehearsed with one rank (graph and inline exchange), exchange-scan timing.
set -o pipefail
TAG=${1:-r3a}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc" >> $O/status; case $rc in 124|134|137|139) exit $rc;; esac; }
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -v -rA --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
chk $? pytest
timeout -k 10 300 python $R/bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
chk $? bench
RLE_BENCH_FORCE_EXCHANGE=1 timeout -k 10 200 python $R/bench.py --steps 20 --warmup 5 --no-cpu --no-north-star --no-concurrent > $O/bench_x_graph.json 2> $O/bench_x_graph.err
chk $? bench_x_graph
RLE_BENCH_FORCE_EXCHANGE=1 RLE_BENCH_GRAPH=0 timeout -k 10 200 python $R/bench.py --steps 20 --warmup 5 --no-cpu --no-north-star --no-concurrent > $O/bench_x_inline.json 2> $O/bench_x_inline.err
chk $? bench_x_inline
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_scan -o run -- python3 $R/tools/dist_scan_prof.py > $O/scan.log 2>&1
chk $? prof_scan
