#!/bin/bash
# CBAA section profile (s_memtime, -DACL_AUCTION_PROF=1 builds) of variants:
# scripts/gpu_sections.sh VARIANT ... (aclswarm_amd/lib/exp/<variant>.so)
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
for v in "$@"; do
  echo "== $v"
  ACLSWARM_AMD_LIB=$PWD/aclswarm_amd/lib/exp/$v.so timeout -k 10 180 python3 scripts/phase_profile.py 2> gpurun_out/sec_$v.err | grep -v amdgpu.ids || { echo "profile $v failed"; tail -20 gpurun_out/sec_$v.err; exit 1; }
done
