#!/bin/bash
set -o pipefail
cd /root/repo
for F in 256 32; do
  echo "formations $F"
  BENCH_ARGS="--formations $F" bash scripts/gpu_ab.sh pf2 noctl streamonly 2>&1 | grep -v "^$" || exit 1
done
