#!/bin/bash
# round 6: the collision list's workgroup counters in 64 groups (rel2) against
# one counter (rel1): C3 headline and the crowded probe; the GPU suite first
set -o pipefail
cd /root/repo
D=gpurun_out/${OUT:-r6_ab_rel}
mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -2 $D/tests.log
for rep in 1 2 3; do
  for v in rel1 rel2; do
    ACLSWARM_AMD_LIB=$PWD/aclswarm_amd/lib/exp/$v.so timeout -k 10 300 python bench.py --no-cpu > $D/c3_${v}_$rep.json 2> $D/c3_${v}_$rep.err || { tail -20 $D/c3_${v}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$D/c3_${v}_$rep.json')); print('$v $rep', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],3), 'ms crowded', round(d['ca_probe']['call_ms'],3), 'ms')" | tee -a $D/summary.txt
  done
done
