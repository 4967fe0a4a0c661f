#!/bin/bash
# C2 full batch, C4 simform500 parity, generator fixtures.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_formation_gen.py -m gpu -x -v --timeout 300 --timeout-method thread -k "c2_full or c4 or n500 or fixtures" > gpurun_out/pytest_c24.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_c24.log; exit 1; }
tail -12 gpurun_out/pytest_c24.log
