#!/bin/bash
# A/B kernel timing over environment settings of the product library: for each "NAME=VAL" (or
# "-" for none) and workload, trace the codec launches and check the round trip.
# usage: bash tools/envab.sh TAG "ENV1 ENV2 ..." [workloads...]
set -o pipefail
TAG=$1; ENVS=$2; shift 2
WLS=${@:-dec64k cfg1}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for E in $ENVS; do
  V=${E//[=\/]/_}
  for WL in $WLS; do
    if [ "$E" = "-" ]; then
      timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/${V}_$WL -o run -- python3 $R/tools/prof_driver.py --workload $WL --reps 5 > $O/${V}_$WL.log 2>&1
    else
      env "$E" timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/${V}_$WL -o run -- python3 $R/tools/prof_driver.py --workload $WL --reps 5 > $O/${V}_$WL.log 2>&1
    fi
    rc=$?; echo "$V $WL rc=$rc $(tail -1 $O/${V}_$WL.log)" >> $O/status
    case $rc in 124|134|137|139) exit $rc;; esac
  done
done
exit 0
