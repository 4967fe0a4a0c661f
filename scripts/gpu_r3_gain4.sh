#!/bin/bash
# GPU tests (in-tree library = new8), then the C4 shard A/B: new6 (one gain
# pass in flight), new7 (four passes in flight in the 1024-thread gain
# kernel), new8 (+ branch-free alignment sums in the wide auction); profile.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
BENCH_ARGS="--config c4 --steps 5 --warmup 2" bash scripts/gpu_r3_iter2.sh new6 new7 new8 || exit 1
ACLSWARM_AMD_LIB=$PWD/aclswarm_amd/lib/exp/wideprof.so timeout -k 10 300 python3 scripts/phase_profile.py --B 2048 --n 500 --L 90 > gpurun_out/phase_wide2.txt 2>&1 || { echo "wide profile failed"; tail -20 gpurun_out/phase_wide2.txt; exit 1; }
cat gpurun_out/phase_wide2.txt
