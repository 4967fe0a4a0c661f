#!/bin/bash
# Interleaved gain-kernel A/B over full bench runs (C3 default workload):
# scripts/gpu_gain_ab.sh variant... (aclswarm_amd/lib/exp/<variant>.so)
set -o pipefail
mkdir -p gpurun_out
cd /root/repo
for rep in 1 2 3; do
  for v in "$@"; do
    ACLSWARM_AMD_LIB=$PWD/aclswarm_amd/lib/exp/$v.so timeout -k 10 240 python3 bench.py --steps 10 --warmup 2 > gpurun_out/gab_$v.json 2> gpurun_out/gab_$v.err || { echo "variant $v failed"; tail -20 gpurun_out/gab_$v.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/gab_$v.json')); r=d['roofline']
print('$v', 'rep $rep', 'value', round(d['value']), r['kernel'], 'avg_launch_ms', round(r['avg_launch_ms'], 4))"
  done
done
