#!/bin/bash
# ADMM (config C5) parity on the first variant, then C5 timing of each variant,
# interleaved twice: scripts/gpu_admm_var.sh V1 V2 ... (aclswarm_amd/lib/exp/V.so)
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
ACLSWARM_AMD_LIB=$PWD/aclswarm_amd/lib/exp/$1.so timeout -k 10 600 python -u -m pytest tests/test_gpu_admm.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_admm_var.log 2>&1 || { echo "admm pytest ($1) failed"; tail -40 gpurun_out/pytest_admm_var.log; exit 1; }
tail -1 gpurun_out/pytest_admm_var.log
for rep in 1 2; do
  for v in "$@"; do
    ACLSWARM_AMD_LIB=$PWD/aclswarm_amd/lib/exp/$v.so timeout -k 10 300 python scripts/admm_bench.py > gpurun_out/admm_$v.json 2> gpurun_out/admm_$v.err || { echo "bench $v failed"; tail -20 gpurun_out/admm_$v.err; exit 1; }
    echo "$v $rep: $(cut -c1-330 gpurun_out/admm_$v.json)"
  done
done
