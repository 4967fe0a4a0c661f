#!/bin/bash
# Device formation generator: GPU parity tests.
set -o pipefail
mkdir -p gpurun_out
cd /root/repo
timeout -k 10 600 python -u -m pytest tests/test_gpu_formation_gen.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gen.log 2>&1 || { echo "generator parity failed"; tail -60 gpurun_out/pytest_gen.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/pytest_gen.log | tail -12
