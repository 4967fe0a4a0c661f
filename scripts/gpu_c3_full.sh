#!/bin/bash
# full-size C3 GPU parity tests, then the C3 bench line with the CA probe (no CPU leg)
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_c3_full.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_c3full.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pytest_c3full.log | head -20; tail -40 gpurun_out/pytest_c3full.log; exit 1; }
grep -E "PASSED|passed" gpurun_out/pytest_c3full.log
timeout -k 10 300 python bench.py --no-cpu --no-setup-ab > gpurun_out/bench_c3p.json 2> gpurun_out/bench_c3p.err || { tail -20 gpurun_out/bench_c3p.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench_c3p.json')); print('value %.0f' % d['value'], 'ms/step %.3f' % d['ms_per_step']); print(d['ca_probe'])"
