#!/bin/bash
# tools/pattern_kinds.py over the product library and every build/variants/librle_*.so, one
# process per build (the pattern kernel of each build timed beside its decode).
#   usage: bash tools/gpu_pattern_variants.sh TAG [workloads] [rounds]
set -o pipefail
TAG=${1:?tag}; WL=${2:-k64_zero,k64_random,dec64k}; RN=${3:-3}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 200 python -u $R/tools/pattern_kinds.py --rounds $RN --workloads $WL > $O/product.jsonl 2> $O/err.log || exit $?
for L in $R/c-filestorage-server-and-client_amd/build/variants/librle_*.so; do
  V=$(basename $L .so); V=${V#librle_}
  RLE_MI355X_LIB=$L timeout -k 10 200 python -u $R/tools/pattern_kinds.py --rounds $RN --workloads $WL > $O/$V.jsonl 2>> $O/err.log || exit $?
done
exit 0
