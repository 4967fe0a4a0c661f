#!/bin/bash
# Round-3 evidence on the final tree: smoke, the C3 bench line (CPU baseline
# included), a rocprofv3 kernel trace of it, HBM-traffic PMC passes (C3, C4),
# the fused kernel's SQ counters, and the C4 / C5 bench lines.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cut -c1-300 gpurun_out/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_c3 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-ca-probe > gpurun_out/prof_c3.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_c3.log; exit 1; }
mkdir -p gpurun_out/prof_c3 && cp $(find /tmp/prof_c3 -name "*kernel_stats.csv" | head -1) gpurun_out/prof_c3/kernel_stats.csv
bash scripts/gpu_pmc.sh || exit 1
rm -rf gpurun_out/pmc_c3 && mv gpurun_out/pmc gpurun_out/pmc_c3
OUT=pmc_fused3 AUCTION_ARGS="--B 65536 --control" bash scripts/gpu_pmc_auction.sh > gpurun_out/pmc_fused3.log 2>&1 || { echo "fused pmc failed"; tail -20 gpurun_out/pmc_fused3.log; exit 1; }
timeout -k 10 600 python bench.py --config c4 --steps 5 --warmup 2 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { echo "bench c4 failed"; tail -30 gpurun_out/bench_c4.err; exit 1; }
cut -c1-300 gpurun_out/bench_c4.json
BENCH_ARGS="--config c4 --no-ca-probe" bash scripts/gpu_pmc.sh || exit 1
rm -rf gpurun_out/pmc_c4 && mv gpurun_out/pmc gpurun_out/pmc_c4
timeout -k 10 600 python bench.py --config c5 --steps 3 --warmup 2 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { echo "bench c5 failed"; tail -30 gpurun_out/bench_c5.err; exit 1; }
cut -c1-300 gpurun_out/bench_c5.json
timeout -k 10 600 python bench.py --config c2 --graph > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { echo "bench c2 failed"; tail -30 gpurun_out/bench_c2.err; exit 1; }
cut -c1-300 gpurun_out/bench_c2.json
