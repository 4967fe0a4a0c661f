#!/bin/bash
# SQ counters of the auction kernel alone (instruction mix, stalls), one
# rocprofv3 pass per counter group, counters only. OUT=<dir under gpurun_out>
# (default pmca). KPAT: the kernels kept (default: the solve kernels).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=${OUT:-pmca}
mkdir -p gpurun_out/$OUT
# pass 0: kernel durations of the same command (kernel trace only), the
# summary's time base for the counters
rm -rf /tmp/pmca_0
timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace -d /tmp/pmca_0 -o run --output-format csv -- \
    python3 scripts/auction_only.py --reps 2 ${AUCTION_ARGS} > gpurun_out/$OUT/out_0.txt 2> gpurun_out/$OUT/err_0.txt || { echo "trace pass failed"; tail -20 gpurun_out/$OUT/err_0.txt; exit 1; }
f=$(find /tmp/pmca_0 -name "*kernel_trace.csv" | head -1)
head -1 "$f" > gpurun_out/$OUT/trace.csv
grep "acl_amd" "$f" >> gpurun_out/$OUT/trace.csv
i=0
for C in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU"; do
  i=$((i+1))
  rm -rf /tmp/pmca_$i
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $C -d /tmp/pmca_$i -o run --output-format csv -- \
      python3 scripts/auction_only.py --reps 2 ${AUCTION_ARGS} > gpurun_out/$OUT/out_$i.txt 2> gpurun_out/$OUT/err_$i.txt || { echo "pmc pass $i failed"; tail -20 gpurun_out/$OUT/err_$i.txt; exit 1; }
  f=$(find /tmp/pmca_$i -name "*counter_collection.csv" | head -1)
  head -1 "$f" > gpurun_out/$OUT/pass_$i.csv
  grep -E "${KPAT:-solve_kernel|auction_kernel|solve_wide_kernel|align_wide_kernel|align_kernel}" "$f" >> gpurun_out/$OUT/pass_$i.csv
done
python3 scripts/pmc_show.py gpurun_out/$OUT
