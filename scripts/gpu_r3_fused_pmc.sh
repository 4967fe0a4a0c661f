#!/bin/bash
# Fused auction + control kernel at C3: phase split (s_memtime stamps), the
# auction alone vs the fused solve, and SQ counters of the fused launch.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/phase_profile.py --B 65536 > gpurun_out/phase_fused.txt 2>&1 || { echo "phase profile failed"; tail -20 gpurun_out/phase_fused.txt; exit 1; }
cat gpurun_out/phase_fused.txt
timeout -k 10 300 python3 scripts/auction_only.py --B 65536 --reps 3 > gpurun_out/ao.txt 2>&1 || { tail -20 gpurun_out/ao.txt; exit 1; }
timeout -k 10 300 python3 scripts/auction_only.py --B 65536 --reps 3 --control >> gpurun_out/ao.txt 2>&1 || { tail -20 gpurun_out/ao.txt; exit 1; }
cat gpurun_out/ao.txt
OUT=pmc_fused AUCTION_ARGS="--B 65536 --control" bash scripts/gpu_pmc_auction.sh
timeout -k 10 900 bash scripts/gpu_admm_pmc.sh > gpurun_out/admm_pmc.log 2>&1 || { echo "admm pmc failed"; tail -20 gpurun_out/admm_pmc.log; exit 1; }
ACLSWARM_AMD_LIB=$PWD/aclswarm_amd/lib/exp/caprof.so timeout -k 10 300 python3 scripts/phase_profile.py --B 65536 --crowd 0.3 > gpurun_out/phase_ca.txt 2>&1 || { echo "ca profile failed"; tail -20 gpurun_out/phase_ca.txt; exit 1; }
cat gpurun_out/phase_ca.txt
