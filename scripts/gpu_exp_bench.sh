#!/bin/bash
# Timing-only comparison of experiment variants (aclswarm_amd/lib/exp/*.so);
# no parity (experiments may read a layout the packer does not write).
set -o pipefail
mkdir -p gpurun_out/exp
cd /root/repo
for so in aclswarm_amd/lib/exp/*.so; do
  nm=$(basename $so .so)
  export ACLSWARM_AMD_LIB=$PWD/$so
  timeout -k 10 300 python bench.py --no-cpu --steps 10 ${BENCH_ARGS} > gpurun_out/exp/bench_$nm.json 2> gpurun_out/exp/bench_$nm.err || { echo "$nm bench failed"; tail -20 gpurun_out/exp/bench_$nm.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/exp/bench_$nm.json')); r=d['roofline']
print('$nm', round(d['value']), 'ms', round(d['ms_per_step'],3), {k:(round(v['avg_launch_ms'],3), round(v['frac'],3)) for k,v in r['kernels'].items()})"
done
