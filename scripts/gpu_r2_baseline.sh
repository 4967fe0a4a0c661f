#!/bin/bash
# Round-2 baseline: phase stamps + SQ counters of the auction kernel.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python3 scripts/phase_profile.py > gpurun_out/phases_base.txt 2>&1 || { echo "phase profile failed"; tail -20 gpurun_out/phases_base.txt; exit 1; }
cat gpurun_out/phases_base.txt
bash scripts/gpu_pmc_auction.sh
python3 scripts/pmc_show.py gpurun_out/pmca
