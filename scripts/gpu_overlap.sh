#!/bin/bash
# Whole-solve time with the auction/gain overlap experiment (ACLSWARM_AMD_OVERLAP
# = number of chunks; 0 = the stream-ordered default), interleaved twice.
set -o pipefail
cd /root/repo
for rep in 1 2; do
  for k in 0 2 4 8; do
    echo -n "overlap=$k rep $rep: "
    ACLSWARM_AMD_OVERLAP=$k timeout -k 10 120 python3 scripts/auction_only.py --B 65536 --reps 3 --control 2> /dev/null || { echo "failed"; exit 1; }
  done
done
