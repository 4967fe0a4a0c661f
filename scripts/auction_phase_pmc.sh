#!/bin/bash
# Per-phase instruction counts of the auction kernel: the diagnostic builds
# aclswarm_amd/lib/exp/stop{0..5}.so (scripts/build_objs.sh stopK
# -DACL_AUCTION_STOP=K) return after phase K; one SQ counter pass each.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=${OUT:-phase_pmc}
mkdir -p gpurun_out/$OUT
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
for k in ${STOPS:-1 2 3 4 5 0}; do
  rm -rf /tmp/pp_$k
  ACLSWARM_AMD_LIB=$PWD/aclswarm_amd/lib/exp/stop$k.so timeout -k 10 -s KILL 120 rocprofv3 --pmc $C -d /tmp/pp_$k -o run --output-format csv -- \
      python3 scripts/auction_only.py --reps 2 ${AO_ARGS} > gpurun_out/$OUT/out_$k.txt 2> gpurun_out/$OUT/err_$k.txt || { echo "pass $k failed"; tail -20 gpurun_out/$OUT/err_$k.txt; exit 1; }
  f=$(find /tmp/pp_$k -name "*counter_collection.csv" | head -1)
  head -1 "$f" > gpurun_out/$OUT/pass_$k.csv
  grep -E "auction_kernel" "$f" >> gpurun_out/$OUT/pass_$k.csv
done
python3 scripts/pmc_show.py gpurun_out/$OUT
