#!/bin/bash
# Round-3 evidence on the final tree (second pass): smoke; C4 HBM-traffic PMC
# passes summarised into profiles/r3c4_pmc_traffic.json before the C4 bench
# line reads it; C3 bench (CPU baseline included) and its kernel trace; C5
# bench and trace; C2 bench; the GPU test suite.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
BENCH_ARGS="--config c4 --no-ca-probe" bash scripts/gpu_pmc.sh || exit 1
rm -rf gpurun_out/pmc_c4 && mv gpurun_out/pmc gpurun_out/pmc_c4
python3 scripts/pmc_summary.py gpurun_out/pmc_c4 gpurun_out/r3c4_pmc_traffic.json > /dev/null && cp gpurun_out/r3c4_pmc_traffic.json profiles/r3c4_pmc_traffic.json
timeout -k 10 600 python bench.py --config c4 --steps 5 --warmup 2 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { echo "bench c4 failed"; tail -30 gpurun_out/bench_c4.err; exit 1; }
cut -c1-200 gpurun_out/bench_c4.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_c4 -o run --output-format csv -- python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu --no-ca-probe > gpurun_out/prof_c4.log 2>&1 || { echo "rocprof c4 failed"; tail -20 gpurun_out/prof_c4.log; exit 1; }
mkdir -p gpurun_out/prof_c4 && cp $(find /tmp/prof_c4 -name "*kernel_stats.csv" | head -1) gpurun_out/prof_c4/kernel_stats.csv
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cut -c1-200 gpurun_out/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_c3 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-ca-probe > gpurun_out/prof_c3.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_c3.log; exit 1; }
mkdir -p gpurun_out/prof_c3 && cp $(find /tmp/prof_c3 -name "*kernel_stats.csv" | head -1) gpurun_out/prof_c3/kernel_stats.csv
timeout -k 10 600 python bench.py --config c5 --steps 3 --warmup 2 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { echo "bench c5 failed"; tail -30 gpurun_out/bench_c5.err; exit 1; }
cut -c1-200 gpurun_out/bench_c5.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_c5 -o run --output-format csv -- python3 bench.py --config c5 --steps 1 --warmup 0 --no-cpu > gpurun_out/prof_c5.log 2>&1 || { echo "c5 prof failed"; tail -20 gpurun_out/prof_c5.log; exit 1; }
mkdir -p gpurun_out/prof_c5 && cp $(find /tmp/prof_c5 -name "*kernel_stats.csv" | head -1) gpurun_out/prof_c5/kernel_stats.csv
timeout -k 10 600 python bench.py --config c2 --graph > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { echo "bench c2 failed"; tail -30 gpurun_out/bench_c2.err; exit 1; }
cut -c1-200 gpurun_out/bench_c2.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu_final.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_final.log
