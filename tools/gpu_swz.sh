set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/tools/ab.sh swz k64_random cfg1 dec64k || exit 1
cd /tmp && export TMPDIR=/tmp
for V in mi355x swz2; do
  if [ $V = mi355x ]; then SO=$R/c-filestorage-server-and-client_amd/librle_mi355x.so; else SO=$R/c-filestorage-server-and-client_amd/build/variants/librle_$V.so; fi
  RLE_MI355X_LIB=$SO timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $R/gpurun_out/swz/pmc_$V/p1 -o run -- python3 $R/tools/prof_driver.py --workload k64_random --reps 3 > $R/gpurun_out/swz/pmc_$V.log 2>&1 || exit 1
done
