#!/bin/bash
# round 6: the persistent workspace (ABI 10: no memset per solve) and the
# per-lane histogram stats; bench with and without --no-persistent, C2 graph
# of 10 steps and C3, after the whole -m gpu suite on the in-tree library
set -o pipefail
cd /root/repo
D=gpurun_out/${OUT:-r6_ab_pers}
mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -2 $D/tests.log
for rep in 1 2 3; do
  for v in pers memset; do
    extra=""; [ $v = memset ] && extra="--no-persistent"
    timeout -k 10 300 python bench.py --no-cpu --no-ca-probe --config c2 --graph --graph-steps 10 $extra > $D/c2_${v}_$rep.json 2> $D/c2_${v}_$rep.err || { tail -20 $D/c2_${v}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$D/c2_${v}_$rep.json')); print('c2 $v $rep', round(d['value']/1e6,3), 'M', round(d['ms_per_step']*1e3,2), 'us')" | tee -a $D/summary.txt
  done
done
for rep in 1 2; do
  for v in pers memset; do
    extra=""; [ $v = memset ] && extra="--no-persistent"
    timeout -k 10 300 python bench.py --no-cpu --no-ca-probe $extra > $D/c3_${v}_$rep.json 2> $D/c3_${v}_$rep.err || { tail -20 $D/c3_${v}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$D/c3_${v}_$rep.json')); print('c3 $v $rep', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],3), 'ms')" | tee -a $D/summary.txt
  done
done
