set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3s_kt
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for WL in m1_zero m1_random m1_runs50; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$WL -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_driver.py --workload $WL --reps 5 --seg > $O/$WL.log 2>&1 || exit $?
done
