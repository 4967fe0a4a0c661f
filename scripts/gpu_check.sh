#!/bin/bash
# One GPU session: parity tests, a short bench, a rocprofv3 kernel-trace profile.
set -o pipefail
mkdir -p gpurun_out
cd /root/repo
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --B 8192 --steps 5 --warmup 1 --no-cpu > gpurun_out/bench_small.json 2> gpurun_out/bench_small.err || { echo "small bench failed"; tail -30 gpurun_out/bench_small.err; exit 1; }
cat gpurun_out/bench_small.json
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
