set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 400 python $R/bench.py > $R/gpurun_out/bench_r1.json 2> $R/gpurun_out/bench_r1.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r1 -o run -- python3 $R/bench.py --steps 20 --no-cpu > $R/gpurun_out/prof_r1.log 2>&1
echo ok
