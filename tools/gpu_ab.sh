#!/bin/bash
# One A/B session on the GPU box (round 5's per-session scripts folded into one): the named GPU
# test modules first, then tools/ab_events.py over the product library and every
# build/variants/librle_*.so (`make -C c-filestorage-server-and-client_amd variant NAME=x DEFS=...`),
# each build's round trip checked before it is timed.
#   usage: bash tools/gpu_ab.sh TAG "tests/test_gpu_parity.py tests/test_gpu_fastpath.py" cfg1,dec64k [--seg]
set -o pipefail
TAG=${1:?tag}
TESTS=${2:-}
WL=${3:-cfg1,dec64k}
SEG=${4:-}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
if [ -n "$TESTS" ]; then
  T=""
  for t in $TESTS; do T="$T $R/$t"; done
  timeout -k 10 900 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> $O/status
  case $rc in 0) ;; *) exit $rc;; esac
fi
timeout -k 10 600 python -u $R/tools/ab_events.py $SEG --workloads $WL --reps 10 --rounds 7 > $O/ab.json 2> $O/ab.err
rc=$?; echo "ab rc=$rc" >> $O/status
exit $rc
