#!/bin/bash
# ADMM C5 kernel-trace summary (rocprofv3 --kernel-trace --stats), REPS batches (default 1)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=${OUT:-admm_prof}
mkdir -p gpurun_out/$OUT
rm -rf /tmp/kt_admm
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/kt_admm -o run --output-format csv -- \
    python3 scripts/admm_bench.py --reps ${REPS:-1} > gpurun_out/$OUT/bench.json 2> gpurun_out/$OUT/err.txt || { tail -20 gpurun_out/$OUT/err.txt; exit 1; }
f=$(find /tmp/kt_admm -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/$OUT/kernel_stats.csv
t=$(find /tmp/kt_admm -name "*kernel_trace.csv" | head -1)
gzip -c "$t" > gpurun_out/$OUT/kernel_trace.csv.gz
cut -d, -f1-4 gpurun_out/$OUT/kernel_stats.csv | cut -c1-150 | head -16
