#!/bin/bash
# Iteration check: GPU tests (PYTEST_K selects), then A/B of library variants
# (aclswarm_amd/lib/exp/<name>.so) on the C3 bench, interleaved twice.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -30; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
if [ $# -gt 0 ]; then bash scripts/gpu_ab.sh "$@"; fi
