#!/bin/bash
# Round-4: decode staging of batches within one residency round (RLE_DEC_CHUNKS 64 / 96 / 128 against
# 192), same process (tools/ab_events.py), the configs[1] batch and its 4 KiB kinds.
# usage: bash tools/gpu_r4s.sh TAG
set -o pipefail
TAG=${1:-r4s}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
timeout -k 10 600 python -u $R/tools/ab_events.py --workloads cfg1,c4k_random,c4k_zero,c4k_runs50,dec64k --reps 40 --rounds 9 > $O/ab.json 2> $O/ab.err
rc=$?; echo "ab rc=$rc" >> $O/status
exit $rc
