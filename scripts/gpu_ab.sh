#!/bin/bash
# Same-box A/B of library variants (aclswarm_amd/lib/exp/<V>.so, built by
# scripts/build_variant.sh), interleaved REPS times (default 2):
#   [TESTS="tests/a.py tests/b.py"] [PYTEST_K=expr] [BENCH_ARGS="--config c4"] [CMD="python3 scripts/auction_only.py ..."] \
#     bash scripts/gpu_ab.sh A B ...
# TESTS: a -m gpu pytest selection run first on the in-tree library (stops on
# failure). Each variant then runs bench.py (--no-cpu --no-ca-probe
# $BENCH_ARGS; one summary line per run) or, with CMD, that command under
# ACLSWARM_AMD_LIB. OUT (required) names the experiment: outputs go to
# gpurun_out/$OUT/ab_<V>_<rep>.*, a fresh directory (an existing one is an
# error, so no run overwrites or mixes with another experiment's files).
set -o pipefail
cd /root/repo
[ -n "$OUT" ] || { echo "OUT=<experiment name> is required"; exit 2; }
D=gpurun_out/$OUT
[ -e "$D" ] && { echo "$D exists: pick a new experiment name"; exit 2; }
mkdir -p "$D"
echo "variants: $* (reps ${REPS:-2})" > "$D/README"
git -C /root/repo log -1 --format=%H >> "$D/README" 2>/dev/null || true
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} $TESTS \
      > $D/ab_tests.log 2>&1 || { tail -40 $D/ab_tests.log; exit 1; }
  tail -2 $D/ab_tests.log
fi
for rep in $(seq 1 ${REPS:-2}); do
  for v in "$@"; do
    lib=$PWD/aclswarm_amd/lib/exp/$v.so
    [ -f "$lib" ] || { echo "missing $lib"; exit 1; }
    if [ -n "$CMD" ]; then
      ACLSWARM_AMD_LIB=$lib timeout -k 10 300 $CMD > $D/ab_${v}_$rep.txt 2>&1 || { echo "$v failed"; tail -20 $D/ab_${v}_$rep.txt; exit 1; }
      echo "$v $rep: $(tail -1 $D/ab_${v}_$rep.txt)" | tee -a "$D/summary.txt"
      continue
    fi
    ACLSWARM_AMD_LIB=$lib timeout -k 10 300 python bench.py --no-cpu --no-ca-probe ${BENCH_ARGS} > $D/ab_${v}_$rep.json 2> $D/ab_${v}_$rep.err || { echo "bench $v failed"; tail -20 $D/ab_${v}_$rep.err; exit 1; }
    python -c "
import json
d = json.load(open('$D/ab_${v}_$rep.json'))
k = d.get('roofline', {}).get('kernels', {})
print('$v', $rep, round(d['value'], 1), d['unit'], round(d['ms_per_step'], 3), 'ms', round(d['roofline']['frac'], 4),
      {n: round(x['avg_launch_ms'], 3) for n, x in k.items() if isinstance(x, dict) and 'avg_launch_ms' in x})" | tee -a "$D/summary.txt"
  done
done
