#!/bin/bash
# ADMM GEMM tile A/B on one box: parity tests (default tile), then C5 at each tile
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_admm.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_admm.log 2>&1 || { echo "admm pytest failed"; tail -40 gpurun_out/pytest_admm.log; exit 1; }
tail -2 gpurun_out/pytest_admm.log
for T in ${TILES:-80 64}; do
  ACLSWARM_AMD_GEMM_TILE=$T timeout -k 10 300 python scripts/admm_bench.py > gpurun_out/admm_bench_t$T.json 2> gpurun_out/admm_bench_t$T.err || { echo "bench $T failed"; tail -20 gpurun_out/admm_bench_t$T.err; exit 1; }
  echo "tile $T: $(cut -c1-400 gpurun_out/admm_bench_t$T.json)"
done
