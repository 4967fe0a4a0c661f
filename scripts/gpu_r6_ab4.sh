#!/bin/bash
# round 6: the CA list release without the per-workgroup fence; its stats
# kernel (per-lane histogram) against the ballot-atomic one (oldstats)
set -o pipefail
cd /root/repo
OUT=r6_ab_nofence REPS=3 BENCH_ARGS="--config c2 --graph --graph-steps 10" bash scripts/gpu_ab.sh nofence oldstats || exit 1
OUT=r6_ab_nofence_c3 REPS=2 bash scripts/gpu_ab.sh nofence oldstats
