#!/bin/bash
# C4 iteration: GPU tests, C4 shard A/B (base vs new), the wide section profile.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
BENCH_ARGS="--config c4 --steps 5 --warmup 2" bash scripts/gpu_r3_iter2.sh base new || exit 1
ACLSWARM_AMD_LIB=$PWD/aclswarm_amd/lib/exp/wideprof.so timeout -k 10 300 python3 scripts/phase_profile.py --B 2048 --n 500 --L 90 > gpurun_out/phase_wide.txt 2>&1 || { echo "wide profile failed"; tail -20 gpurun_out/phase_wide.txt; exit 1; }
cat gpurun_out/phase_wide.txt
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_c5 -o run --output-format csv -- python3 bench.py --config c5 --steps 1 --warmup 0 --no-cpu > gpurun_out/prof_c5.log 2>&1 || { echo "c5 prof failed"; tail -20 gpurun_out/prof_c5.log; exit 1; }
mkdir -p gpurun_out/prof_c5 && cp $(find /tmp/prof_c5 -name "*kernel_stats.csv" | head -1) gpurun_out/prof_c5/kernel_stats.csv
cut -d, -f1-4 gpurun_out/prof_c5/kernel_stats.csv | head -25
