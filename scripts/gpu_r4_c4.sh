#!/bin/bash
# Round 4, C4: the wide solve as alignment + 512-thread auction launches.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_c4_full.py tests/test_gpu_parity.py tests/test_gpu_episode.py tests/test_gpu_admm.py tests/test_gpu_facade.py > gpurun_out/r4_c4t.log 2>&1 || { tail -40 gpurun_out/r4_c4t.log; exit 1; }
tail -3 gpurun_out/r4_c4t.log
BENCH_ARGS="--config c4" bash scripts/gpu_ab.sh w1 w2
