#!/bin/bash
# Compare experiment variants (aclswarm_amd/lib/exp/*.so): solve parity tests
# against each, then a short bench; per-kernel times.
set -o pipefail
mkdir -p gpurun_out/exp
cd /root/repo
for so in aclswarm_amd/lib/exp/*.so; do
  nm=$(basename $so .so)
  export ACLSWARM_AMD_LIB=$PWD/$so
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/exp/pytest_$nm.log 2>&1 || { echo "$nm parity failed"; tail -40 gpurun_out/exp/pytest_$nm.log; exit 1; }
  timeout -k 10 300 python bench.py --no-cpu --steps 10 ${BENCH_ARGS} > gpurun_out/exp/bench_$nm.json 2> gpurun_out/exp/bench_$nm.err || { echo "$nm bench failed"; tail -20 gpurun_out/exp/bench_$nm.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/exp/bench_$nm.json')); r=d['roofline']
print('$nm', round(d['value']), 'ms', round(d['ms_per_step'],3), {k:(round(v['avg_launch_ms'],3), round(v['frac'],3)) for k,v in r['kernels'].items()})"
  tail -1 gpurun_out/exp/pytest_$nm.log
done
