#!/bin/bash
# GPU tests (in-tree library), then the C4 shard A/B: base (full column
# write-back) vs new (changed who entries only).
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
BENCH_ARGS="--config c4 --steps 5 --warmup 2" bash scripts/gpu_r3_iter2.sh base new || exit 1
