#!/bin/bash
# Pair-symmetric gain kernel: all GPU tests, then the bench with and without it.
set -o pipefail
mkdir -p gpurun_out
cd /root/repo
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_pair.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/pytest_pair.log; exit 1; }
tail -2 gpurun_out/pytest_pair.log
for mode in 1 0; do
  ACLSWARM_AMD_GAIN_PAIR=$mode timeout -k 10 300 python bench.py --no-cpu --steps 10 > gpurun_out/bench_pair$mode.json 2> gpurun_out/bench_pair$mode.err || { echo "bench $mode failed"; tail -20 gpurun_out/bench_pair$mode.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/bench_pair$mode.json')); r=d['roofline']
print('pair=$mode', round(d['value']), 'ms', round(d['ms_per_step'],3), {k:(round(v['avg_launch_ms'],3), round(v['frac'],3)) for k,v in r['kernels'].items()})"
done
