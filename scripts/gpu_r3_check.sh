#!/bin/bash
# GPU tests + smoke + the C3 and C5 bench lines (round 3 iteration check).
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -30; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
grep -cE "PASSED" gpurun_out/pytest_gpu.log; tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cut -c1-1500 gpurun_out/bench.json
timeout -k 10 600 python bench.py --config c5 --steps 3 --warmup 2 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { echo "bench c5 failed"; tail -30 gpurun_out/bench_c5.err; exit 1; }
cut -c1-2500 gpurun_out/bench_c5.json
