#!/bin/bash
# One GPU session: parity tests, phase profile, bench.
set -o pipefail
mkdir -p gpurun_out
cd /root/repo
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python scripts/phase_profile.py > gpurun_out/phases.txt 2>&1 || { echo "phase profile failed"; tail -30 gpurun_out/phases.txt; exit 1; }
cat gpurun_out/phases.txt
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
