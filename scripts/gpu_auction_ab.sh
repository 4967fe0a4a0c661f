#!/bin/bash
# Auction-only A/B of library variants on one box, interleaved twice:
# scripts/gpu_auction_ab.sh A B ... (aclswarm_amd/lib/exp/{A,B}.so)
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
for rep in 1 2; do
  for v in "$@"; do
    echo -n "$v $rep: "
    ACLSWARM_AMD_LIB=$PWD/aclswarm_amd/lib/exp/$v.so timeout -k 10 120 python3 scripts/auction_only.py --B 65536 --reps 3 ${AUCTION_ARGS} 2> gpurun_out/aab_$v.err || { echo "variant $v failed"; tail -20 gpurun_out/aab_$v.err; exit 1; }
  done
done
