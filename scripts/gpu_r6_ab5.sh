#!/bin/bash
# round 6: ADMM post-process writing the next iteration's Pm (no pm launch per
# iteration) against the tree before; the ADMM GPU tests first
set -o pipefail
cd /root/repo
OUT=${OUT:-r6_ab_c5pm} REPS=3 TESTS="tests/test_gpu_admm.py tests/test_gpu_codegen.py tests/test_gpu_facade.py" BENCH_ARGS="--config c5" \
  bash scripts/gpu_ab.sh ${VARS:-c5base c5pm}
[ -n "$PROF" ] && OUT=$PROF REPS=2 bash scripts/gpu_admm_prof.sh
exit 0
