#!/bin/bash
# round 6: stats kernel with DPP wave sums and readlane bins (stats1) against
# the shuffle version (stats0), C2 graph of 10 steps; stats + fused tests first
set -o pipefail
cd /root/repo
OUT=${OUT:-r6_ab_stats} REPS=3 TESTS="tests/test_gpu_stats.py tests/test_gpu_fused.py" BENCH_ARGS="--config c2 --graph --graph-steps 10" \
  bash scripts/gpu_ab.sh stats0 stats1
