#!/bin/bash
# round 6: new-path GPU tests (trials, central episodes, fused parity), the
# Eigen-rule risk count over 65 536 C3 swarms, then the A/B of the fused
# kernel's prefetch variants (scripts/gpu_ab.sh, C3 bench lines).
set -o pipefail
cd /root/repo
OUT=r6_new1 RISK_S=65536 bash scripts/gpu_r6_new.sh || exit 1
OUT=r6_ab_pref REPS=3 TESTS="tests/test_gpu_fused.py tests/test_gpu_c3_full.py" bash scripts/gpu_ab.sh ab_base ab_x3 ab_x34
