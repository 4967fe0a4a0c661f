#!/bin/bash
# auction block-size variants: parity tests of every auction path, then the C2 and C3 bench lines
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_margins.py tests/test_gpu_episode.py tests/test_gpu_facade.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_small.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pytest_small.log | head -20; tail -40 gpurun_out/pytest_small.log; exit 1; }
tail -2 gpurun_out/pytest_small.log
for c in c2 c3; do
  timeout -k 10 300 python bench.py --config $c --no-cpu --no-setup-ab > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { tail -20 gpurun_out/bench_$c.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/bench_$c.json')); r=d['roofline']
print('$c', 'value %.0f' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'call_ms %.4f' % r['pipeline']['call_ms'], {k:round(v['avg_launch_ms'],4) for k,v in r['kernels'].items()})"
done
