#!/bin/bash
# round 5: episodes run their auctions with skip_margin (ep1) vs with the margin (ep0), n = 100 and n = 20
set -o pipefail
cd /root/repo
OUT=r5_ab_ep TESTS="-m gpu tests/test_gpu_episode.py" CMD="python3 scripts/episode_bench.py --no-cpu" bash scripts/gpu_ab.sh ep0 ep1 && \
OUT=r5_ab_ep20 CMD="python3 scripts/episode_bench.py --no-cpu --n 20 --B 4096" bash scripts/gpu_ab.sh ep0 ep1
