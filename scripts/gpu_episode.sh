#!/bin/bash
# Closed-loop episodes: GPU parity tests, then the episode bench.
set -o pipefail
mkdir -p gpurun_out
cd /root/repo
timeout -k 10 600 python -u -m pytest tests/test_gpu_episode.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_episode.log 2>&1 || { echo "episode parity failed"; tail -60 gpurun_out/pytest_episode.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/pytest_episode.log | tail -10
if [ -f scripts/episode_bench.py ]; then
  timeout -k 10 300 python scripts/episode_bench.py > gpurun_out/episode_bench.json 2> gpurun_out/episode_bench.err || { echo "episode bench failed"; tail -30 gpurun_out/episode_bench.err; exit 1; }
  cat gpurun_out/episode_bench.json
fi
