#!/bin/bash
# round 5 final measurements: PART=tests|bench|prof (default tests bench)
#   tests: the whole -m gpu suite; bench: bench.py default (C3) / c4 / c5 / c2 --graph;
#   prof: rocprofv3 kernel-trace + PMC traffic + SQ passes (scripts/gpu_profile_round.sh, ROUND=r5)
set -o pipefail
cd /root/repo
O=gpurun_out/r5_final
mkdir -p $O
for p in ${PART:-tests bench}; do
  case $p in
    tests)
      timeout -k 10 1100 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ \
          > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
      tail -3 $O/tests.log ;;
    bench)
      timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
      timeout -k 10 300 python bench.py --config c4 --no-cpu > $O/bench_c4.json 2> $O/bench_c4.err || { tail -20 $O/bench_c4.err; exit 1; }
      timeout -k 10 300 python bench.py --config c5 > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
      timeout -k 10 300 python bench.py --config c2 --graph --no-cpu > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
      for f in default c4 c5 c2; do python -c "
import json; d=json.load(open('$O/bench_$f.json'))
print('$f', round(d['value'],1), d['unit'], round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],4), 'margin', d.get('margin',{}).get('value_margin_on'))"; done ;;
    prof)
      ROUND=r5 bash scripts/gpu_profile_round.sh c3 c4 c5 || exit 1 ;;
  esac
done
