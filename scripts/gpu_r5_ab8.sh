#!/bin/bash
# round 5: LDS-DMA staging of the untransposed GEMMs (gdma) vs register staging (g11), C5
set -o pipefail
cd /root/repo
OUT=r5_ab_c5dma TESTS="-m gpu tests/test_gpu_admm.py tests/test_gpu_codegen.py" BENCH_ARGS="--config c5" bash scripts/gpu_ab.sh g11 gdma
