#!/bin/bash
# round 5: sparse wide columns with per-vehicle exception counts (C4), margin-cost split (C3)
set -o pipefail
cd /root/repo
OUT=r5_ab_c4b TESTS="-m gpu tests" BENCH_ARGS="--config c4" bash scripts/gpu_ab.sh base sp2 || exit 1
OUT=r5_ab_marg REPS=1 bash scripts/gpu_ab.sh cl nomarg noselm noall || exit 1
mkdir -p gpurun_out/r5_c4prof
ACLSWARM_AMD_LIB=$PWD/aclswarm_amd/lib/exp/wprof.so timeout -k 10 300 python scripts/phase_profile.py --n 500 --B 2048 > gpurun_out/r5_c4prof/phase_sparse.txt 2>&1
tail -20 gpurun_out/r5_c4prof/phase_sparse.txt
