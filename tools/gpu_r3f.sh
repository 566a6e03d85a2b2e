#!/bin/bash
# r3f: periodic decode tiles + uniform encode tiles: full GPU parity, bench, kernel trace per kind.
set -o pipefail
TAG=${1:-r3f}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc" >> $O/status; case $rc in 124|134|137|139) exit $rc;; esac; [ $rc -ne 0 ] && exit $rc; }
timeout -k 10 700 python -u -m pytest $R/tests -m gpu -x -v -rA --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
chk $? pytest
timeout -k 10 300 python $R/bench.py --steps 20 --warmup 5 --no-cpu > $O/bench.json 2> $O/bench.err
chk $? bench
cd /tmp && export TMPDIR=/tmp
for WL in cfg1 dec64k k64_random k64_zero k64_runs50 k64_runs90; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$WL -o run -- python3 $R/tools/prof_driver.py --workload $WL --reps 5 > $O/kt_$WL.log 2>&1
  chk $? kt_$WL
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_scan -o run -- python3 $R/tools/dist_scan_prof.py > $O/scan.log 2>&1
chk $? prof_scan
cd $R
timeout -k 10 500 python $R/tools/e2e_compare.py --reps 3 > $O/e2e.json 2> $O/e2e.err
chk $? e2e
