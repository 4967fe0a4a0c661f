#!/bin/bash
# Round-3 full check: GPU tests, smoke, C3 bench (with CPU baseline), C5 bench,
# C4 shard bench, and a rocprofv3 kernel trace of the C3 bench.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -30; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
grep -cE "PASSED" gpurun_out/pytest_gpu.log; tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -3 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cut -c1-1500 gpurun_out/bench.json
timeout -k 10 600 python bench.py --config c5 --steps 3 --warmup 2 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { echo "bench c5 failed"; tail -30 gpurun_out/bench_c5.err; exit 1; }
cut -c1-800 gpurun_out/bench_c5.json
timeout -k 10 600 python bench.py --config c4 --steps 5 --warmup 2 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { echo "bench c4 failed"; tail -30 gpurun_out/bench_c4.err; exit 1; }
cut -c1-800 gpurun_out/bench_c4.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-ca-probe > gpurun_out/prof_c3.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_c3.log; exit 1; }
find gpurun_out/prof_c3 -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'cut -d, -f1-8 {} | head -12'
