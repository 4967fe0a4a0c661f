#!/bin/bash
# round 6: the new GPU tests (central-assignment episodes, trials), then the
# Eigen-rule risk count over the bench's C3 workload (RISK_S swarms).
#   OUT=<dir> [RISK_S=65536] bash scripts/gpu_r6_new.sh
set -o pipefail
cd /root/repo
[ -n "$OUT" ] || { echo "OUT=<name> is required"; exit 2; }
D=gpurun_out/$OUT
mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_trial.py tests/test_gpu_episode.py -k "trial or central" \
    > $D/tests.log 2>&1 || { tail -60 $D/tests.log; exit 1; }
tail -3 $D/tests.log
if [ -n "$RISK_S" ]; then
  timeout -k 10 600 python -u scripts/eigen_variant_risk.py --S $RISK_S --threads 16 \
      > $D/eigen_variant_risk.json 2> $D/eigen_variant_risk.err || { tail -20 $D/eigen_variant_risk.err; exit 1; }
  cat $D/eigen_variant_risk.json
fi
