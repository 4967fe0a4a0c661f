#!/bin/bash
# round 5: GEMM operand loads through global pointers, transform/zero-fill at the LDS store (agl) vs adiag, C5
set -o pipefail
cd /root/repo
OUT=r5_ab_c5gl TESTS="-m gpu tests/test_gpu_admm.py" BENCH_ARGS="--config c5" bash scripts/gpu_ab.sh agb agl
