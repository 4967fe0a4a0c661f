#!/bin/bash
# GPU tests, price/margin A/B, the wide-kernel phase profile, and the
# episode bench (eager and as a replayed HIP graph) at n = 100 and n = 20.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
bash scripts/gpu_r3_iter2.sh base new nomargin || exit 1
ACLSWARM_AMD_LIB=$PWD/aclswarm_amd/lib/exp/wideprof.so timeout -k 10 300 python3 scripts/phase_profile.py --B 2048 --n 500 --L 90 > gpurun_out/phase_wide.txt 2>&1 || { echo "wide profile failed"; tail -20 gpurun_out/phase_wide.txt; exit 1; }
cat gpurun_out/phase_wide.txt
timeout -k 10 300 python3 scripts/episode_bench.py --graph > gpurun_out/episode_c3.json 2> gpurun_out/episode_c3.err || { echo "episode failed"; tail -20 gpurun_out/episode_c3.err; exit 1; }
cut -c1-600 gpurun_out/episode_c3.json
timeout -k 10 300 python3 scripts/episode_bench.py --graph --n 20 --B 4096 --no-cpu > gpurun_out/episode_c2.json 2> gpurun_out/episode_c2.err || { echo "episode c2 failed"; tail -20 gpurun_out/episode_c2.err; exit 1; }
cut -c1-600 gpurun_out/episode_c2.json
timeout -k 10 300 python3 scripts/hungarian_bench.py > gpurun_out/hungarian.json 2> gpurun_out/hungarian.err || { echo "hungarian failed"; tail -20 gpurun_out/hungarian.err; exit 1; }
cut -c1-600 gpurun_out/hungarian.json
