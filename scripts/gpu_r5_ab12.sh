#!/bin/bash
# round 5 (diagnostic): the crowded C3 solve with the CA pair kernel's f64 atan2/asin/cos/sin
# (cabase) vs f32 stand-ins (cadiag: wrong results, a bound on what the library calls cost)
set -o pipefail
cd /root/repo
OUT=r5_ab_cadiag CMD="python3 scripts/auction_only.py --B 65536 --control --crowd 0.3 --reps 3" bash scripts/gpu_ab.sh cabase cadiag
