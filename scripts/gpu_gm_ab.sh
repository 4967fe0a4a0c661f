#!/bin/bash
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_margins.py tests/test_gpu_episode.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gm.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pytest_gm.log | head -20; tail -30 gpurun_out/pytest_gm.log; exit 1; }
tail -1 gpurun_out/pytest_gm.log
bash scripts/gpu_ab.sh base gm
