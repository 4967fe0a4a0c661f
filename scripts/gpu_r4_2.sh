#!/bin/bash
# Round 4: same-box A/B of the fused control phase (base = round 3, new1 =
# first rewrite, new2 = LDS constants fixed, new3 = 24-bit index multiplies) and SQ counters per phase
# (stop builds) of new2.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_ab.sh base new1 new2 new3 || exit 1
O=gpurun_out/r4_phase
mkdir -p $O
C1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES"
run() {  # name lib args
  local name=$1 lib=$2 args=$3
  rm -rf /tmp/pp_$name
  ACLSWARM_AMD_LIB=$lib timeout -k 10 -s KILL 150 rocprofv3 --pmc $C1 -d /tmp/pp_$name -o run --output-format csv -- \
      python3 scripts/auction_only.py --B 65536 --reps 2 $args > $O/out_$name.txt 2> $O/err_$name.txt || { echo "pass $name failed"; tail -20 $O/err_$name.txt; exit 1; }
  f=$(find /tmp/pp_$name -name "*counter_collection.csv" | head -1)
  head -1 "$f" > $O/pass_$name.csv
  grep -E "auction_kernel" "$f" >> $O/pass_$name.csv
}
for k in 3 4 5; do run s$k $PWD/aclswarm_amd/lib/exp/stop$k.so ""; done
run auc $PWD/aclswarm_amd/lib/exp/new3.so ""
run fused $PWD/aclswarm_amd/lib/exp/new3.so "--control"
python3 scripts/pmc_show.py $O
