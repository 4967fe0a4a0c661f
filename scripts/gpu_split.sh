#!/bin/bash
# per-kernel times with and without overlap
set -o pipefail
mkdir -p gpurun_out
cd /root/repo
for S in 1 0; do
  ACL_SERIAL=$S timeout -k 10 300 python bench.py --no-cpu --steps 5 > gpurun_out/bench_s$S.json 2> gpurun_out/bench_s$S.err || { echo "bench failed"; tail -20 gpurun_out/bench_s$S.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/bench_s$S.json'))
print('serial=$S value', round(d['value']), 'ms/step', round(d['ms_per_step'],2)); r=d['roofline']
print({k:(round(v['avg_launch_ms'],3), round(v['frac'],3)) for k,v in r['kernels'].items()})"
done
