#!/bin/bash
# SQ/TA counters of one kernel of the solve (KERNEL=gain_kernel|solve_kernel|...),
# one rocprofv3 pass per counter group, counters only.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
K=${KERNEL:-gain_kernel}
mkdir -p gpurun_out/pmck
i=0
for C in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
         "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_IFETCH" \
         "TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  rm -rf /tmp/pmck_$i
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $C -d /tmp/pmck_$i -o run --output-format csv -- \
      python3 scripts/auction_only.py --B 16384 --reps 2 --control > gpurun_out/pmck/out_$i.txt 2> gpurun_out/pmck/err_$i.txt || { echo "pmc pass $i failed"; tail -20 gpurun_out/pmck/err_$i.txt; exit 1; }
  f=$(find /tmp/pmck_$i -name "*counter_collection.csv" | head -1)
  head -1 "$f" > gpurun_out/pmck/pass_$i.csv
  grep "$K" "$f" >> gpurun_out/pmck/pass_$i.csv || true
done
wc -l gpurun_out/pmck/*.csv
