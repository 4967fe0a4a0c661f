#!/bin/bash
# C5 A/B of library variants (aclswarm_amd/lib/exp/<v>.so), with the ADMM
# GPU tests run against each non-base variant first.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" != base ]; then
    ACLSWARM_AMD_LIB=$PWD/aclswarm_amd/lib/exp/$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_admm.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_admm_$v.log 2>&1 || { echo "pytest $v failed"; tail -30 gpurun_out/pytest_admm_$v.log; exit 1; }
    echo "$v: $(tail -1 gpurun_out/pytest_admm_$v.log)"
  fi
done
for rep in 1 2; do
  for v in "$@"; do
    ACLSWARM_AMD_LIB=$PWD/aclswarm_amd/lib/exp/$v.so timeout -k 10 300 python bench.py --config c5 --steps 2 --warmup 1 --no-cpu > gpurun_out/c5_${v}_$rep.json 2> gpurun_out/c5_${v}_$rep.err || { echo "c5 $v failed"; tail -20 gpurun_out/c5_${v}_$rep.err; exit 1; }
    python -c "
import json;d=json.load(open('gpurun_out/c5_${v}_$rep.json'))
print('$v', $rep, round(d['value'],1), round(d['ms_per_step'],2), round(d['roofline']['frac'],4))"
  done
done
