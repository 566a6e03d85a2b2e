#!/bin/bash
# HBM traffic (FETCH_SIZE, WRITE_SIZE; one rocprofv3 --pmc pass each) of the decode, the pattern
# kernel and the copy on dec64k, for the product library and build/variants/librle_pal128.so.
#   usage: bash tools/gpu_pattern_pmc.sh TAG
set -o pipefail
TAG=${1:?tag}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for V in product pal128; do
  if [ $V = product ]; then unset RLE_MI355X_LIB; else export RLE_MI355X_LIB=$R/c-filestorage-server-and-client_amd/build/variants/librle_$V.so; fi
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/p_${V}_$C -o run -- python3 $R/tools/pattern_kinds.py --workloads dec64k --reps 5 > $O/${V}_$C.log 2>&1 || exit $?
  done
done
exit 0
