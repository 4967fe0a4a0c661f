#!/bin/bash
# round 6 final measurements: PART="tests bench prof" (default tests bench)
#   tests: the whole -m gpu suite + __graft_entry__.smoke(); bench: bench.py default (C3) / c4 /
#   c5 / c2 --graph, and the trial line; prof: C3 rocprofv3 kernel trace, PMC traffic, SQ passes
set -o pipefail
cd /root/repo
O=gpurun_out/${OUT:-r6_final}
mkdir -p $O
for p in ${PART:-tests bench}; do
  case $p in
    tests)
      timeout -k 10 1100 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ \
          > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
      tail -3 $O/tests.log
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
      tail -1 $O/smoke.log ;;
    bench)
      timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
      timeout -k 10 300 python bench.py --config c4 --no-cpu > $O/bench_c4.json 2> $O/bench_c4.err || { tail -20 $O/bench_c4.err; exit 1; }
      timeout -k 10 300 python bench.py --config c5 > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
      timeout -k 10 300 python bench.py --config c2 --graph --graph-steps 10 --no-cpu > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
      for f in default c4 c5 c2; do python -c "
import json; d=json.load(open('$O/bench_$f.json'))
print('$f', round(d['value'],1), d['unit'], round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],4), 'margin', d.get('margin',{}).get('value_margin_on'), 'crowded', d.get('ca_probe',{}).get('call_ms'))"; done ;;
    prof)
      OUT=r6f_c3_prof bash scripts/gpu_prof.sh || exit 1
      OUT=r6f_c3_pmc bash scripts/gpu_pmc.sh || exit 1
      OUT=r6f_c3_sq AUCTION_ARGS="--B 65536 --n 100 --control" bash scripts/gpu_pmc_auction.sh || exit 1 ;;
  esac
done
