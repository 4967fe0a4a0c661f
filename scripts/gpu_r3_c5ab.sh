#!/bin/bash
# ADMM iteration: ADMM GPU tests, then the C5 bench A/B (base vs new), interleaved.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_admm.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_admm.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_admm.log; exit 1; }
tail -2 gpurun_out/pytest_admm.log
for rep in 1 2; do
  for v in base new; do
    ACLSWARM_AMD_LIB=$PWD/aclswarm_amd/lib/exp/$v.so timeout -k 10 300 python bench.py --config c5 --steps 2 --warmup 1 --no-cpu > gpurun_out/c5_${v}_$rep.json 2> gpurun_out/c5_${v}_$rep.err || { echo "c5 $v failed"; tail -20 gpurun_out/c5_${v}_$rep.err; exit 1; }
    python -c "
import json;d=json.load(open('gpurun_out/c5_${v}_$rep.json'))
print('$v', $rep, round(d['value'],1), round(d['ms_per_step'],2), round(d['roofline']['frac'],4))"
  done
done
