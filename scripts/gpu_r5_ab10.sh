#!/bin/bash
# round 5: LDS-DMA staging for every transpose combination (gdma3) vs untransposed only (gdma2), C5
set -o pipefail
cd /root/repo
OUT=r5_ab_c5dma3 TESTS="-m gpu tests/test_gpu_admm.py tests/test_gpu_codegen.py" BENCH_ARGS="--config c5" bash scripts/gpu_ab.sh gdma2 gdma3
