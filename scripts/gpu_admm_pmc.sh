#!/bin/bash
# PMC passes over the ADMM C5 batch (GEMM kernels): MFMA busy, L2 hit rate, HBM bytes
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/admm_pmc
mkdir -p $O
i=0
for C in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES" \
         "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  rm -rf /tmp/apmc_$i
  timeout -k 10 -s KILL 180 rocprofv3 --pmc $C -d /tmp/apmc_$i -o run --output-format csv -- \
      python3 scripts/admm_bench.py --reps 1 > $O/out_$i.txt 2> $O/err_$i.txt || { echo "pmc pass $i failed"; tail -20 $O/err_$i.txt; exit 1; }
  f=$(find /tmp/apmc_$i -name "*counter_collection.csv" | head -1)
  head -1 "$f" > $O/pass_$i.csv
  grep "gemm" "$f" >> $O/pass_$i.csv
done
ls -la $O
