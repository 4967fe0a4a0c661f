#!/bin/bash
# Variant study of the fused auction kernel: for each library
# aclswarm_amd/lib/exp/<name>.so, the C3 auction alone (and the fused solve
# with CTRL=1) timed and counted (SQ_INSTS_VALU/SALU, VALU-active, wave
# cycles): scripts/gpu_variants.sh OUT name...
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift
mkdir -p $OUT
ARGS="--B 65536"
[ "${CTRL:-0}" = 1 ] && ARGS="$ARGS --control"
C1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES"
for v in "$@"; do
  ACLSWARM_AMD_LIB=$PWD/aclswarm_amd/lib/exp/$v.so timeout -k 10 150 python3 scripts/auction_only.py $ARGS --reps 5 > $OUT/time_$v.txt 2>&1 || { echo "time $v failed"; tail -5 $OUT/time_$v.txt; exit 1; }
  echo "$v $(tail -1 $OUT/time_$v.txt)"
done
for v in "$@"; do
  rm -rf /tmp/pv_$v
  ACLSWARM_AMD_LIB=$PWD/aclswarm_amd/lib/exp/$v.so timeout -k 10 -s KILL 150 rocprofv3 --pmc $C1 -d /tmp/pv_$v -o run --output-format csv -- \
      python3 scripts/auction_only.py $ARGS --reps 2 > $OUT/out_$v.txt 2> $OUT/err_$v.txt || { echo "pmc $v failed"; tail -20 $OUT/err_$v.txt; exit 1; }
  f=$(find /tmp/pv_$v -name "*counter_collection.csv" | head -1)
  head -1 "$f" > $OUT/pass_$v.csv
  grep -E "auction_kernel" "$f" >> $OUT/pass_$v.csv
done
python3 scripts/pmc_show.py $OUT
