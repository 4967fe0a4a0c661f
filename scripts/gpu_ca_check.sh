#!/bin/bash
# collision-avoidance path: parity tests that exercise it, full-size crowded C3, the bench CA probe
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c3_full.py tests/test_gpu_episode.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_ca.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pytest_ca.log | head -20; tail -40 gpurun_out/pytest_ca.log; exit 1; }
tail -1 gpurun_out/pytest_ca.log
timeout -k 10 300 python bench.py --no-cpu --no-setup-ab > gpurun_out/bench_ca.json 2> gpurun_out/bench_ca.err || { tail -20 gpurun_out/bench_ca.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench_ca.json')); print('value %.0f' % d['value'], 'ms/step %.3f' % d['ms_per_step']); print(d['ca_probe'])"
