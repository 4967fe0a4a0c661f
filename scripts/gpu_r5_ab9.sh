#!/bin/bash
# round 5: LDS-DMA staging of the untransposed GEMMs with the operand transform on the landed pieces (gdma2) vs without (gdma), C5
set -o pipefail
cd /root/repo
OUT=r5_ab_c5dma2 TESTS="-m gpu tests/test_gpu_admm.py tests/test_gpu_codegen.py" BENCH_ARGS="--config c5" bash scripts/gpu_ab.sh gdma gdma2
