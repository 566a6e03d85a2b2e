#!/bin/bash
# Quick GPU check: the -m gpu parity suite (stop at first failure), then optional extra steps.
# usage: bash tools/gpu_check.sh TAG [timeline] [probe]
set -o pipefail
TAG=${1:-chk}; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for step in "$@"; do
  case $step in
    timeline)
      for w in cfg1 c4k_random c4k_zero; do
        RLE_MI355X_LIB=$R/c-filestorage-server-and-client_amd/build/variants/librle_tl.so timeout -k 10 120 python $R/tools/timeline.py --workload $w > $O/tl_$w.txt 2>&1
        rc=$?; echo "timeline $w rc=$rc" >> $O/status; [ $rc -ne 0 ] && exit $rc
      done;;
    probe)
      timeout -k 10 60 $R/build/dispatch_probe > $O/dispatch.txt 2>&1
      rc=$?; echo "probe rc=$rc" >> $O/status; [ $rc -ne 0 ] && exit $rc;;
    kt)
      cd /tmp && export TMPDIR=/tmp
      for w in cfg1 dec64k; do
        timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$w -o run -- python3 $R/tools/prof_driver.py --workload $w --reps 5 > $O/kt_$w.log 2>&1
        rc=$?; echo "kt $w rc=$rc" >> $O/status; [ $rc -ne 0 ] && exit $rc
      done
      cd $R;;
  esac
done
exit 0
