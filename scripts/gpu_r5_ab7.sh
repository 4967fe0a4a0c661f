#!/bin/bash
# round 5: GEMM K-loop variants (C5) and the wide kernel's table reads with explicit address spaces (C4)
set -o pipefail
cd /root/repo
OUT=r5_ab_c5loop TESTS="-m gpu tests/test_gpu_admm.py" BENCH_ARGS="--config c5" bash scripts/gpu_ab.sh g00 g01 g11 && \
OUT=r5_ab_c4as TESTS="-m gpu tests/test_gpu_parity.py tests/test_gpu_c4_full.py" BENCH_ARGS="--config c4" bash scripts/gpu_ab.sh agb r5n
