#!/bin/bash
# Same-box A/B of library variants (aclswarm_amd/lib/exp/<V>.so, built by
# scripts/build_variant.sh), interleaved REPS times (default 2):
#   [TESTS="tests/a.py tests/b.py"] [PYTEST_K=expr] [BENCH_ARGS="--config c4"] [CMD="python3 scripts/auction_only.py ..."] \
#     bash scripts/gpu_ab.sh A B ...
# TESTS: a -m gpu pytest selection run first on the in-tree library (stops on
# failure). Each variant then runs bench.py (--no-cpu --no-ca-probe
# $BENCH_ARGS; one summary line per run) or, with CMD, that command under
# ACLSWARM_AMD_LIB. Outputs under gpurun_out/ab_<V>_<rep>.*
set -o pipefail
mkdir -p gpurun_out
cd /root/repo
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} $TESTS \
      > gpurun_out/ab_tests.log 2>&1 || { tail -40 gpurun_out/ab_tests.log; exit 1; }
  tail -2 gpurun_out/ab_tests.log
fi
for rep in $(seq 1 ${REPS:-2}); do
  for v in "$@"; do
    lib=$PWD/aclswarm_amd/lib/exp/$v.so
    [ -f "$lib" ] || { echo "missing $lib"; exit 1; }
    if [ -n "$CMD" ]; then
      ACLSWARM_AMD_LIB=$lib timeout -k 10 300 $CMD > gpurun_out/ab_${v}_$rep.txt 2>&1 || { echo "$v failed"; tail -20 gpurun_out/ab_${v}_$rep.txt; exit 1; }
      echo "$v $rep: $(tail -1 gpurun_out/ab_${v}_$rep.txt)"
      continue
    fi
    ACLSWARM_AMD_LIB=$lib timeout -k 10 300 python bench.py --no-cpu --no-ca-probe ${BENCH_ARGS} > gpurun_out/ab_${v}_$rep.json 2> gpurun_out/ab_${v}_$rep.err || { echo "bench $v failed"; tail -20 gpurun_out/ab_${v}_$rep.err; exit 1; }
    python -c "
import json
d = json.load(open('gpurun_out/ab_${v}_$rep.json'))
k = d.get('roofline', {}).get('kernels', {})
print('$v', $rep, round(d['value'], 1), d['unit'], round(d['ms_per_step'], 3), 'ms', round(d['roofline']['frac'], 4),
      {n: round(x['avg_launch_ms'], 3) for n, x in k.items() if isinstance(x, dict) and 'avg_launch_ms' in x})"
  done
done
