#!/bin/bash
# GPU tests (in-tree library), then the C4 shard A/B: base (levels one at a
# time) vs new (levels in pairs); then the wide auction's SQ counters.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
BENCH_ARGS="--config c4 --steps 5 --warmup 2" bash scripts/gpu_r3_iter2.sh base new || exit 1
OUT=pmc_wide AUCTION_ARGS="--B 2048 --n 500 --L 90" bash scripts/gpu_pmc_auction.sh > gpurun_out/pmc_wide.log 2>&1 || { tail -20 gpurun_out/pmc_wide.log; exit 1; }
tail -30 gpurun_out/pmc_wide.log
