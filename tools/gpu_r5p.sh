#!/bin/bash
# Round 5 (r5p): issue-order A/B for the large decode batch (heavy / light blocks alternating per
# workgroup block or per wave, index order) and the staging swizzle, same process; the two-kind
# batch k64_z50 (zero / runs50) tells whether a store-bound kind overlaps a run-heavy one.
#   usage: bash tools/gpu_r5p.sh TAG
set -o pipefail
TAG=${1:-r5p}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
hostname > $O/host.txt
timeout -k 10 600 python -u $R/tools/ab_events.py --workloads dec64k,k64_z50,k64_zero,k64_runs50,k64_runs90,k64_random --reps 6 --rounds 5 > $O/ab.json 2> $O/ab.err
rc=$?; echo "ab rc=$rc" >> $O/status
exit $rc
