#!/bin/bash
# ADMM (C5) parity and timing per GEMM tile setting on one library build:
# LIBV=<variant> TILES="80 81" scripts/gpu_admm_tiles.sh
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
[ -n "$LIBV" ] && export ACLSWARM_AMD_LIB=$PWD/aclswarm_amd/lib/exp/$LIBV.so
for T in ${TILES:-80 81}; do
  ACLSWARM_AMD_GEMM_TILE=$T timeout -k 10 600 python -u -m pytest tests/test_gpu_admm.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_admm_t$T.log 2>&1 || { echo "admm pytest (tile $T) failed"; tail -30 gpurun_out/pytest_admm_t$T.log; exit 1; }
  echo "tile $T: $(tail -n 1 gpurun_out/pytest_admm_t$T.log)"
done
for rep in 1 2; do
  for T in ${TILES:-80 81}; do
    ACLSWARM_AMD_GEMM_TILE=$T timeout -k 10 300 python scripts/admm_bench.py > gpurun_out/admm_t$T.json 2> gpurun_out/admm_t$T.err || { echo "bench $T failed"; tail -20 gpurun_out/admm_t$T.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/admm_t$T.json')); print('tile $T rep $rep:', round(d['ms_per_batch'], 1), 'ms', round(d['value']), 'formations/s', d['iters_xy'], d['iters_z'])"
  done
done
