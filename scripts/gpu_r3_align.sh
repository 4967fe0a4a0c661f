#!/bin/bash
# Alignment as its own launch: all GPU tests, then C3 and C2 A/B (base vs new).
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
bash scripts/gpu_r3_iter2.sh base new || exit 1
BENCH_ARGS="--config c2" bash scripts/gpu_ab.sh base new || exit 1
