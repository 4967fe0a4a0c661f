#!/bin/bash
# round 6: the 128-thread (n <= 32) auction instantiation built for 6 / 7 / 8
# waves per SIMD (C2: 4 096 swarms, 12 / 14 / 14 resident per CU)
set -o pipefail
cd /root/repo
OUT=${OUT:-r6_ab_occ} REPS=3 TESTS="tests/test_gpu_parity.py" PYTEST_K="c2 or swarm6 or simform20" BENCH_ARGS="--config c2 --graph --graph-steps 10" \
  bash scripts/gpu_ab.sh occ6 occ7 occ8
