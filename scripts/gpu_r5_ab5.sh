#!/bin/bash
# round 5: ADMM symmetric GEMM, diagonal tiles as 15 upper blocks (adiag) vs HEAD (abase), C5
set -o pipefail
cd /root/repo
OUT=r5_ab_c5diag TESTS="-m gpu tests/test_gpu_admm.py" BENCH_ARGS="--config c5" bash scripts/gpu_ab.sh abase adiag
