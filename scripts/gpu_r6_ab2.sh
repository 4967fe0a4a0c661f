#!/bin/bash
# round 6: the 16-byte atan table rows (C3) and the prefetching stats kernel
# with one event pair around the graph replays (C2), against the tree before
set -o pipefail
cd /root/repo
OUT=r6_ab_atan REPS=3 TESTS="-m gpu tests/" \
  bash scripts/gpu_ab.sh ab_base st4 || exit 1
OUT=r6_ab_c2g REPS=2 BENCH_ARGS="--config c2 --graph" bash scripts/gpu_ab.sh ab_base st4 || exit 1
OUT=r6_ab_c2g10 REPS=2 BENCH_ARGS="--config c2 --graph --graph-steps 10" bash scripts/gpu_ab.sh st4
