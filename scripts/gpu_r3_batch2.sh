#!/bin/bash
# All GPU tests, the C5 A/B (ADMM norm fused into w_kernel), the C3 A/B
# (multi-workgroup swarm statistics), then the default bench line and a
# rocprofv3 kernel trace of it.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -30; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for rep in 1 2; do
  for v in base new; do
    ACLSWARM_AMD_LIB=$PWD/aclswarm_amd/lib/exp/$v.so timeout -k 10 300 python bench.py --config c5 --steps 2 --warmup 1 --no-cpu > gpurun_out/c5_${v}_$rep.json 2> gpurun_out/c5_${v}_$rep.err || { echo "c5 $v failed"; tail -20 gpurun_out/c5_${v}_$rep.err; exit 1; }
    python -c "
import json;d=json.load(open('gpurun_out/c5_${v}_$rep.json'))
print('c5', '$v', $rep, round(d['value'],1), round(d['ms_per_step'],2), round(d['roofline']['frac'],4))"
  done
done
bash scripts/gpu_ab.sh base new || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cut -c1-600 gpurun_out/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_c3 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-ca-probe > gpurun_out/prof_c3.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_c3.log; exit 1; }
mkdir -p gpurun_out/prof_c3 && cp $(find /tmp/prof_c3 -name "*kernel_stats.csv" | head -1) gpurun_out/prof_c3/kernel_stats.csv
cut -d, -f1-4 gpurun_out/prof_c3/kernel_stats.csv | head -8
