#!/bin/bash
# native swarm statistics: GPU tests, then the C2 and C3 bench lines (no CPU leg)
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_stats.py tests/test_abi.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_stats.log 2>&1 || { tail -40 gpurun_out/pytest_stats.log; exit 1; }
tail -2 gpurun_out/pytest_stats.log
for c in c2 c3; do
  timeout -k 10 300 python bench.py --config $c --no-cpu --no-setup-ab > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { tail -20 gpurun_out/bench_$c.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/bench_$c.json')); r=d['roofline']
print('$c', 'value %.0f' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'call_ms %.4f' % r['pipeline']['call_ms'])"
done
