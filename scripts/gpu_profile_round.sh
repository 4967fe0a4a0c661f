#!/bin/bash
# One round's committed profiles, parameterised: ROUND=r4 bash scripts/gpu_profile_round.sh [c3] [c4] [c5]
# per config: rocprofv3 --kernel-trace --stats of bench.py (gpu_prof.sh),
# the two HBM traffic PMC passes (gpu_pmc.sh), and the SQ counter passes of
# the fused solve (gpu_pmc_auction.sh); c5: the ADMM kernel trace
# (gpu_admm_prof.sh). Outputs under gpurun_out/${ROUND}_<cfg>_*; summarise
# with scripts/pmc_summary.py / pmc_auction_summary.py into profiles/.
set -o pipefail
cd /root/repo
ROUND=${ROUND:-r4}
CFGS=${*:-c3 c4}
for c in $CFGS; do
  case $c in
    c3) BA=""; AA="--B 65536 --n 100 --control" ;;
    c4) BA="--config c4"; AA="--B 2048 --n 500 --L 90 --control" ;;
    c5) bash scripts/gpu_admm_prof.sh || exit 1; continue ;;
    *) echo "unknown config $c"; exit 1 ;;
  esac
  OUT=${ROUND}_${c}_prof BENCH_ARGS="$BA" bash scripts/gpu_prof.sh || exit 1
  OUT=${ROUND}_${c}_pmc BENCH_ARGS="$BA" bash scripts/gpu_pmc.sh || exit 1
  OUT=${ROUND}_${c}_sq AUCTION_ARGS="$AA" bash scripts/gpu_pmc_auction.sh || exit 1
done
