#!/bin/bash
# rocprofv3 kernel trace + stats of the bench (kernel-trace only: no PMC here).
# STEPS / WARMUP (default 5 / 1): the bench's timed and untimed steps.
set -o pipefail
cd /root/repo
OUT=${OUT:-prof}
mkdir -p /tmp/$OUT gpurun_out/$OUT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/$OUT -o run --output-format csv -- python3 bench.py --steps ${STEPS:-5} --warmup ${WARMUP:-1} --no-cpu --no-ca-probe ${BENCH_ARGS} > gpurun_out/$OUT/bench_out.json 2> gpurun_out/$OUT/rocprof.err || { echo "rocprof failed"; tail -30 gpurun_out/$OUT/rocprof.err; exit 1; }
for f in $(find /tmp/$OUT -name "*kernel_stats.csv"); do cp $f gpurun_out/$OUT/kernel_stats.csv; done
# per-dispatch durations of our kernels only
for f in $(find /tmp/$OUT -name "*kernel_trace.csv"); do head -1 $f > gpurun_out/$OUT/acl_dispatches.csv; grep "acl_amd" $f >> gpurun_out/$OUT/acl_dispatches.csv; done
grep -E "Name|acl_amd" gpurun_out/$OUT/kernel_stats.csv | cut -c1-300
cat gpurun_out/$OUT/bench_out.json | cut -c1-300
