#!/bin/bash
# auction kernel iteration: GPU parity tests of the auction paths, then
# auction-only timings (new vs old kernel) and the phase stamps.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_margins.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_auction.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" gpurun_out/pytest_auction.log | head -30; tail -60 gpurun_out/pytest_auction.log; exit 1; }
tail -2 gpurun_out/pytest_auction.log
timeout -k 10 120 python scripts/auction_only.py --B 65536 --reps 3 || exit 1
timeout -k 10 120 python scripts/phase_profile.py || exit 1
