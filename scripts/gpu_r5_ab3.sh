#!/bin/bash
# round 5: C3 successor-test factor and publication rounds; C4 sparse v3 time and HBM traffic
set -o pipefail
cd /root/repo
OUT=r5_ab_c3b TESTS="-m gpu tests" bash scripts/gpu_ab.sh cl gf pr2 pr4 || exit 1
OUT=r5_ab_c4c BENCH_ARGS="--config c4" bash scripts/gpu_ab.sh base sp3 || exit 1
for v in base sp3; do
  ACLSWARM_AMD_LIB=$PWD/aclswarm_amd/lib/exp/$v.so OUT=r5_c4pmc_$v BENCH_ARGS="--config c4" bash scripts/gpu_pmc.sh || exit 1
done
