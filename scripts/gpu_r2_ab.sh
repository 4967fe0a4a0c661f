#!/bin/bash
# GPU parity suite on the in-tree library, then an interleaved auction-only A/B
# of experiment variants: scripts/gpu_r2_ab.sh [variant ...]
# (aclswarm_amd/lib/exp/<variant>.so; PYTEST_K narrows the suite, SKIP_TESTS=1 skips it)
set -o pipefail
mkdir -p gpurun_out
cd /root/repo
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_ab.log 2>&1 || { echo "parity failed"; grep -E "FAIL|Error|error" gpurun_out/pytest_ab.log | head -20; tail -40 gpurun_out/pytest_ab.log; exit 1; }
  tail -3 gpurun_out/pytest_ab.log
fi
if [ $# -gt 0 ]; then scripts/gpu_auction_ab.sh "$@"; fi
