set -o pipefail
TAG=${1:-r6be}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R && timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_segmented.py tests/test_gpu_parity.py > $O/pytest.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
for WL in m1_random m1_runs50 mixed; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pf_$WL -o run -- python3 $R/tools/prof_driver.py --workload $WL --seg --warm 5 --reps 10 > $O/pf_$WL.log 2>&1 || exit $?
  RLE_MI355X_LIB=$R/c-filestorage-server-and-client_amd/build/variants/librle_nophasefree.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/np_$WL -o run -- python3 $R/tools/prof_driver.py --workload $WL --seg --warm 5 --reps 10 > $O/np_$WL.log 2>&1 || exit $?
done
