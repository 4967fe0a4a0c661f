#!/bin/bash
# round 6: C2 step timeline after the stats change, then diagnostic bounds of
# the fused control phase's formation-distance and atan terms (C3 bench lines)
set -o pipefail
cd /root/repo
OUT=r6_c2trace2 bash scripts/gpu_r6_c2trace.sh || exit 1
OUT=r6_ab_diag REPS=3 bash scripts/gpu_ab.sh ab_base d_nodstar d_noatan
