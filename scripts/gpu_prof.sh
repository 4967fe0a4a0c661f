#!/bin/bash
# rocprofv3 kernel trace + stats of the bench (kernel-trace only: no PMC here).
set -o pipefail
cd /root/repo
mkdir -p /tmp/prof gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu ${BENCH_ARGS} > gpurun_out/prof/bench_out.json 2> gpurun_out/prof/rocprof.err || { echo "rocprof failed"; tail -30 gpurun_out/prof/rocprof.err; exit 1; }
for f in $(find /tmp/prof -name "*kernel_stats.csv"); do cp $f gpurun_out/prof/kernel_stats.csv; done
# per-dispatch durations of our kernels only
for f in $(find /tmp/prof -name "*kernel_trace.csv"); do head -1 $f > gpurun_out/prof/acl_dispatches.csv; grep "acl_amd" $f >> gpurun_out/prof/acl_dispatches.csv; done
grep -E "Name|acl_amd" gpurun_out/prof/kernel_stats.csv | cut -c1-300
cat gpurun_out/prof/bench_out.json | cut -c1-300
