#!/bin/bash
# GPU tests (in-tree library), C4 shard A/B (new3: column-major who table,
# new5: 8x8 tiles), C5 A/B (new5 vs new6: the LDS Cholesky), wide profile.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
BENCH_ARGS="--config c4 --steps 5 --warmup 2" bash scripts/gpu_r3_iter2.sh new3 new5 || exit 1
bash scripts/gpu_r3_c5ab2.sh new5 new6 || exit 1
ACLSWARM_AMD_LIB=$PWD/aclswarm_amd/lib/exp/wideprof.so timeout -k 10 300 python3 scripts/phase_profile.py --B 2048 --n 500 --L 90 > gpurun_out/phase_wide2.txt 2>&1 || { echo "wide profile failed"; tail -20 gpurun_out/phase_wide2.txt; exit 1; }
cat gpurun_out/phase_wide2.txt
