#!/bin/bash
# round 6: stats-kernel change -- its tests, then C2 (graph) and C3 bench lines.
set -o pipefail
cd /root/repo
D=gpurun_out/${OUT:-r6_c2}
mkdir -p $D
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_stats.py tests/test_gpu_parity.py -k "stats or c2" > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -2 $D/tests.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py --config c2 --graph --no-cpu --no-ca-probe > $D/c2_graph_$rep.json 2> $D/c2_graph_$rep.err || { tail -20 $D/c2_graph_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$D/c2_graph_$rep.json')); print('c2 graph', round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,1), 'us', round(d['roofline']['call_ms']*1e3,1), 'us call')"
done
timeout -k 10 300 python bench.py --config c2 --no-cpu --no-ca-probe > $D/c2_eager.json 2> $D/c2_eager.err || { tail -20 $D/c2_eager.err; exit 1; }
python -c "import json; d=json.load(open('$D/c2_eager.json')); print('c2 eager', round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,1), 'us')"
