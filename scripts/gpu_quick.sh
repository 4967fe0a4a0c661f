#!/bin/bash
# quick GPU iteration: solve parity tests + auction-only timing + bench
set -o pipefail
mkdir -p gpurun_out
cd /root/repo
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_parity.log 2>&1 || { echo "parity failed"; tail -50 gpurun_out/pytest_parity.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/pytest_parity.log | tail -40
timeout -k 10 120 python scripts/auction_only.py --B 65536 --reps 3 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python scripts/phase_profile.py 2>&1 | grep -v amdgpu.ids | head -9
timeout -k 10 600 python bench.py --no-cpu ${BENCH_ARGS} > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { echo "bench failed"; tail -30 gpurun_out/bench_quick.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench_quick.json'))
print('value', d['value'], 'ms/step', d['ms_per_step']); r=d['roofline']
print({k:(v['avg_launch_ms'], v['frac']) for k,v in r['kernels'].items()}, 'pipeline', r['pipeline']['call_ms'], r['pipeline']['frac'])"
