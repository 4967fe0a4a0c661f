#!/bin/bash
# Comparator (acl_hungarian_batch): GPU parity tests, bench, rocprofv3 stats.
set -o pipefail
mkdir -p gpurun_out
cd /root/repo
timeout -k 10 600 python -u -m pytest tests/test_gpu_hungarian.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_hung.log 2>&1 || { echo "hungarian parity failed"; tail -60 gpurun_out/pytest_hung.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/pytest_hung.log | tail -30
timeout -k 10 300 python scripts/hungarian_bench.py > gpurun_out/hung_bench.json 2> gpurun_out/hung_bench.err || { echo "bench failed"; tail -30 gpurun_out/hung_bench.err; exit 1; }
cat gpurun_out/hung_bench.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_hung -o hung -- python3 scripts/hungarian_bench.py --reps 3 --cpu-budget 1 > gpurun_out/hung_prof.log 2>&1 || { echo "rocprof failed"; tail -30 gpurun_out/hung_prof.log; exit 1; }
find gpurun_out/prof_hung -name "*kernel_stats.csv" | head -3
