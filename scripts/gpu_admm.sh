#!/bin/bash
# ADMM GPU session: parity tests, then the C5 timing.
set -o pipefail
mkdir -p gpurun_out
cd /root/repo
timeout -k 10 600 python -u -m pytest tests/test_gpu_admm.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_admm.log 2>&1 || { echo "admm pytest failed"; tail -60 gpurun_out/pytest_admm.log; exit 1; }
tail -15 gpurun_out/pytest_admm.log
timeout -k 10 300 python scripts/admm_bench.py ${ADMM_ARGS} > gpurun_out/admm_bench.json 2> gpurun_out/admm_bench.err || { echo "admm bench failed"; tail -30 gpurun_out/admm_bench.err; exit 1; }
cat gpurun_out/admm_bench.json
