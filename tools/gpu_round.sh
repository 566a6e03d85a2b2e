#!/bin/bash
# Full GPU round: parity tests (incl. e2e), bench, host-path bench, rocprofv3 kernel trace of the
# bench and PMC traffic passes for the bench workload.   usage: bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-round}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
timeout -k 10 900 python -u -m pytest $R/tests -m gpu -v -rA --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -u -m pytest $R/tests/test_e2e_server.py -m gpu -s -q --timeout 240 --timeout-method thread > $O/e2e.log 2>&1
rc=$?; echo "e2e rc=$rc" >> $O/status
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 400 python $R/bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc" >> $O/status
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python $R/tools/hostpath_bench.py > $O/hostpath.json 2> $O/hostpath.err
rc=$?; echo "hostpath rc=$rc" >> $O/status
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 500 python -u $R/tools/roofline_sweep.py > $O/sweep.json 2> $O/sweep.err
rc=$?; echo "sweep rc=$rc" >> $O/status
case $rc in 124|134|137|139) exit $rc;; esac
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 20 --no-cpu --no-concurrent > $O/prof.log 2>&1
rc=$?; echo "prof rc=$rc" >> $O/status
case $rc in 124|134|137|139) exit $rc;; esac
for WL in cfg1 dec64k; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 240 rocprofv3 --pmc $C --output-format csv -d $O/pmc_${WL}_$C -o run -- python3 $R/tools/prof_driver.py --workload $WL --reps 3 > $O/pmc_${WL}_$C.log 2>&1
    rc=$?; echo "pmc $WL $C rc=$rc" >> $O/status
    case $rc in 124|134|137|139) exit $rc;; esac
  done
done
