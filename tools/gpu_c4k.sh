#!/bin/bash
# GPU parity suite, then kernel traces of configs[1] beside its one-kind halves and two 64 KiB kinds.
# usage: bash tools/gpu_c4k.sh TAG [workloads...]   (default: cfg1 c4k_random c4k_zero k64_random k64_zero)
set -o pipefail
TAG=${1:-c4k}; shift
WLS=${@:-cfg1 c4k_random c4k_zero k64_random k64_zero}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
for WL in $WLS; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$WL -o run -- python3 $R/tools/prof_driver.py --workload $WL --reps 10 > $O/kt_$WL.log 2>&1
  rc=$?; echo "kt $WL rc=$rc" >> $O/status; [ $rc -ne 0 ] && exit $rc
done
exit 0
