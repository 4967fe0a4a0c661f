#!/bin/bash
# round 6: collision-avoidance kernels scan the swarm masks (no list, no
# memset) + wave-reduced stats: the whole GPU suite, then same-box bench
# lines old (ab_x3) vs new (r6_scan) for C2 (graph) and C3 with the crowded probe.
set -o pipefail
cd /root/repo
D=gpurun_out/${OUT:-r6_scan}
mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ \
    > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -2 $D/tests.log
for rep in 1 2; do
  for v in ab_x3 r6_scan; do
    lib=$PWD/aclswarm_amd/lib/exp/$v.so
    ACLSWARM_AMD_LIB=$lib timeout -k 10 300 python bench.py --config c2 --graph --no-cpu --no-ca-probe > $D/c2_${v}_$rep.json 2> $D/c2_${v}_$rep.err || { tail -20 $D/c2_${v}_$rep.err; exit 1; }
    ACLSWARM_AMD_LIB=$lib timeout -k 10 300 python bench.py --no-cpu > $D/c3_${v}_$rep.json 2> $D/c3_${v}_$rep.err || { tail -20 $D/c3_${v}_$rep.err; exit 1; }
    python -c "
import json
a=json.load(open('$D/c2_${v}_$rep.json')); b=json.load(open('$D/c3_${v}_$rep.json'))
print('$v', $rep, 'c2', round(a['value']/1e6,2), 'M', round(a['ms_per_step']*1e3,1), 'us | c3', round(b['value']/1e6,3), 'M', round(b['ms_per_step'],3), 'ms | crowded', round(b['ca_probe']['call_ms'],2), 'ms')" | tee -a $D/summary.txt
  done
done
