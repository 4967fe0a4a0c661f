#!/bin/bash
# Per-phase VALU/SALU/LDS instruction counts of the auction (stop builds,
# scripts/build_objs.sh stopK -DACL_AUCTION_STOP=K) and of the fused launch,
# with the VALU mix by type where the counters exist.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/phase_pmc3
mkdir -p $O
timeout -k 10 -s KILL 120 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
MIX=""
for c in SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT64; do
  grep -q "\b$c\b" $O/avail.txt && MIX="$MIX $c"
done
echo "mix counters:$MIX"
C1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES"
run() {  # name lib args counters
  local name=$1 lib=$2 args=$3 cs=$4
  rm -rf /tmp/pp_$name
  ACLSWARM_AMD_LIB=$lib timeout -k 10 -s KILL 120 rocprofv3 --pmc $cs -d /tmp/pp_$name -o run --output-format csv -- \
      python3 scripts/auction_only.py --reps 2 $args > $O/out_$name.txt 2> $O/err_$name.txt || { echo "pass $name failed"; tail -20 $O/err_$name.txt; exit 1; }
  f=$(find /tmp/pp_$name -name "*counter_collection.csv" | head -1)
  head -1 "$f" > $O/pass_$name.csv
  grep -E "auction_kernel" "$f" >> $O/pass_$name.csv
}
for k in 1 2 3 4 5 0; do
  run s$k $PWD/aclswarm_amd/lib/exp/stop$k.so "" "$C1"
  if [ -n "$MIX" ]; then run m$k $PWD/aclswarm_amd/lib/exp/stop$k.so "" "$MIX"; fi
done
run fused $PWD/aclswarm_amd/lib/libaclswarm_amd.so "--control" "$C1"
if [ -n "$MIX" ]; then run mfused $PWD/aclswarm_amd/lib/libaclswarm_amd.so "--control" "$MIX"; fi
python3 scripts/pmc_show.py $O
