#!/bin/bash
# Fused auction + control kernel: GPU tests, the C3 bench line, a kernel trace.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -30; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
grep -cE "PASSED" gpurun_out/pytest_gpu.log; tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py --no-cpu ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cut -c1-4000 gpurun_out/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fused -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-ca-probe > gpurun_out/prof_fused.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_fused.log; exit 1; }
find gpurun_out/prof_fused -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'cut -d, -f1-8 {} | head -12'
