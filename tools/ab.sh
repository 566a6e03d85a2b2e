#!/bin/bash
# A/B kernel timing: for each experimental build in build/variants/librle_*.so (and the product
# library), trace the codec launches of the given workloads and check the round trip.
# usage: bash tools/ab.sh TAG [workloads...]     (default: dec64k cfg1)
set -o pipefail
TAG=${1:-ab}; shift
WLS=${@:-dec64k cfg1}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for SO in $R/c-filestorage-server-and-client_amd/librle_mi355x.so $R/c-filestorage-server-and-client_amd/build/variants/librle_*.so; do
  V=$(basename $SO .so)
  for WL in $WLS; do
    RLE_MI355X_LIB=$SO timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/${V}_$WL -o run -- python3 $R/tools/prof_driver.py --workload $WL --reps 5 > $O/${V}_$WL.log 2>&1
    rc=$?; echo "$V $WL rc=$rc $(tail -1 $O/${V}_$WL.log)" >> $O/status
    case $rc in 124|134|137|139) exit $rc;; esac   # rc 1 = round-trip mismatch (diagnostic builds)
  done
done
exit 0
