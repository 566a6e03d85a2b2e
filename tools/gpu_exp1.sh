#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/exp1; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for PAD in 0 128 4224; do
  RLE_BENCH_PAD=$PAD timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/pad${PAD}_zero -o run -- python3 $R/tools/prof_driver.py --workload k64_zero --reps 5 > $O/pad$PAD.log 2>&1 || exit $?
  RLE_BENCH_PAD=$PAD timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/pad${PAD}_random -o run -- python3 $R/tools/prof_driver.py --workload k64_random --reps 5 >> $O/pad$PAD.log 2>&1 || exit $?
done
bash $R/tools/ab.sh exp1ab k64_zero k64_random
