#!/bin/bash
# A/B of library variants on the same box: scripts/gpu_ab.sh A B ...
# (aclswarm_amd/lib/exp/{A,B}.so), interleaved twice; BENCH_ARGS extra flags.
set -o pipefail
mkdir -p gpurun_out
cd /root/repo
for rep in 1 2; do
  for v in "$@"; do
    ACLSWARM_AMD_LIB=$PWD/aclswarm_amd/lib/exp/$v.so timeout -k 10 300 python bench.py --no-cpu --no-ca-probe ${BENCH_ARGS} > gpurun_out/ab_${v}_$rep.json 2> gpurun_out/ab_${v}_$rep.err || { echo "bench $v failed"; tail -20 gpurun_out/ab_${v}_$rep.err; exit 1; }
    python -c "
import json;d=json.load(open('gpurun_out/ab_${v}_$rep.json'));k=d['roofline']['kernels']
print('$v', $rep, round(d['value']), round(d['roofline']['frac'], 4), {n: round(x['avg_launch_ms'], 3) for n, x in k.items()})"
  done
done
