#!/bin/bash
# round 5: sparse wide columns v4 (C4) vs the dense table
set -o pipefail
cd /root/repo
OUT=r5_ab_c4d TESTS="-m gpu tests/test_gpu_parity.py tests/test_gpu_c4_full.py tests/test_gpu_fused.py tests/test_gpu_episode.py" BENCH_ARGS="--config c4" bash scripts/gpu_ab.sh base sp4 && \
  bash scripts/gpu_r5_ab5.sh
