#!/bin/bash
# round 5: ca_pair_kernel occupancy bound 4 (base: 128 VGPRs, 21 spilled to scratch) / 3 / 2 waves per SIMD, crowded C3 solve
set -o pipefail
cd /root/repo
OUT=r5_ab_caocc CMD="python3 scripts/auction_only.py --B 65536 --control --crowd 0.3 --reps 3" bash scripts/gpu_ab.sh ca4 ca3 ca2
