#!/bin/bash
# Collision avoidance by pairs: GPU tests, then the crowded probe same-box
# against the previous library (aclswarm_amd/lib/exp/base.so), then the
# fused-kernel profiling of scripts/gpu_r3_fused_pmc.sh.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -30; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for rep in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export ACLSWARM_AMD_LIB=$PWD/aclswarm_amd/lib/exp/base.so; else unset ACLSWARM_AMD_LIB; fi
    timeout -k 10 300 python bench.py --no-cpu --steps 5 --warmup 1 > gpurun_out/ca_${v}_$rep.json 2> gpurun_out/ca_${v}_$rep.err || { echo "bench $v failed"; tail -20 gpurun_out/ca_${v}_$rep.err; exit 1; }
    python -c "
import json;d=json.load(open('gpurun_out/ca_${v}_$rep.json'));c=d['ca_probe']
print('$v', $rep, round(d['value']), 'probe', round(c['call_ms'],3), {k: round(x,3) for k,x in c['kernel_ms'].items()}, c['ca_active_swarms'], c['ca_vehicles'])"
  done
done
unset ACLSWARM_AMD_LIB
bash scripts/gpu_r3_fused_pmc.sh
