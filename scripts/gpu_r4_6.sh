#!/bin/bash
# Round 4: binade atan, cheaper margin publication (new5) -- parity of the
# n <= 128 kernels, section profile, same-box A/B against new3 / new4.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_margins.py tests/test_gpu_fused.py tests/test_gpu_c3_full.py tests/test_gpu_facade.py tests/test_gpu_formats.py tests/test_gpu_episode.py tests/test_gpu_stats.py > gpurun_out/r4_t6.log 2>&1 || { tail -40 gpurun_out/r4_t4.log; exit 1; }
tail -3 gpurun_out/r4_t6.log


bash scripts/gpu_ab.sh new5 new6
