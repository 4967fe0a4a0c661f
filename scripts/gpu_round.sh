#!/bin/bash
# Full GPU pass: every -m gpu test, smoke(), the default bench line, the
# rocprofv3 kernel-trace/stats pass and the two PMC traffic passes.
set -o pipefail
mkdir -p gpurun_out
cd /root/repo
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
grep -cE "PASSED" gpurun_out/pytest_gpu.log; tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
bash scripts/gpu_prof.sh && bash scripts/gpu_pmc.sh
