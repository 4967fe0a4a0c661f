#!/bin/bash
# round 5: Newton-Schulz GEMM launches gated on the last step's count of parts still iterating (gq1) vs not (gq0), C5
set -o pipefail
cd /root/repo
OUT=r5_ab_c5gate TESTS="-m gpu tests/test_gpu_admm.py tests/test_gpu_codegen.py" BENCH_ARGS="--config c5" bash scripts/gpu_ab.sh gq0 gq1
