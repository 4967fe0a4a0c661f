#!/bin/bash
# round 6: the whole -m gpu suite on the in-tree library, then (optional)
# the Eigen-rule risk count over the bench's C3 workload.
#   OUT=<dir> [RISK=1] bash scripts/gpu_r6_check.sh
set -o pipefail
cd /root/repo
[ -n "$OUT" ] || { echo "OUT=<name> is required"; exit 2; }
D=gpurun_out/$OUT
mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ \
    > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -2 $D/tests.log
if [ -n "$RISK" ]; then
  timeout -k 10 600 python -u scripts/eigen_variant_risk.py --S ${RISK_S:-16384} --threads 16 \
      > $D/eigen_variant_risk.json 2> $D/eigen_variant_risk.err || { tail -20 $D/eigen_variant_risk.err; exit 1; }
  cat $D/eigen_variant_risk.json
fi
