#!/bin/bash
# HBM traffic (FETCH_SIZE / WRITE_SIZE passes) of the C3 and C4 bench kernels,
# and SQ counters of the wide auction at C4.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
bash scripts/gpu_pmc.sh || exit 1
mv gpurun_out/pmc gpurun_out/pmc_c3
BENCH_ARGS="--config c4 --no-ca-probe" bash scripts/gpu_pmc.sh || exit 1
mv gpurun_out/pmc gpurun_out/pmc_c4
OUT=pmc_wide AUCTION_ARGS="--B 2048 --n 500 --L 90" bash scripts/gpu_pmc_auction.sh || exit 1
