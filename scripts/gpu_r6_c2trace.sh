#!/bin/bash
# round 6: C2 step timeline (rocprofv3 kernel trace of bench.py --config c2
# --graph, every dispatch kept) for the launch-overhead work.
set -o pipefail
cd /root/repo
OUT=${OUT:-r6_c2trace}
mkdir -p /tmp/$OUT gpurun_out/$OUT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats -d /tmp/$OUT -o run --output-format csv -- python3 bench.py --config c2 --graph --steps 10 --warmup 2 --no-cpu --no-ca-probe > gpurun_out/$OUT/bench_out.json 2> gpurun_out/$OUT/rocprof.err || { echo "rocprof failed"; tail -30 gpurun_out/$OUT/rocprof.err; exit 1; }
for f in $(find /tmp/$OUT -name "*kernel_stats.csv"); do cp $f gpurun_out/$OUT/kernel_stats.csv; done
for f in $(find /tmp/$OUT -name "*kernel_trace.csv"); do cp $f gpurun_out/$OUT/kernel_trace.csv; done
for f in $(find /tmp/$OUT -name "*memory_copy_trace.csv"); do cp $f gpurun_out/$OUT/memory_copy_trace.csv; done
cut -c1-200 gpurun_out/$OUT/kernel_stats.csv | head -20
