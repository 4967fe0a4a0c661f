#!/bin/bash
# round 6: trial bench smoke (small B), then the C3-shape trial line (both
# assignment modes) and the episode CBAA-vs-central comparison.
set -o pipefail
cd /root/repo
D=gpurun_out/${OUT:-r6_trials}
mkdir -p $D
timeout -k 10 300 python -u scripts/episode_bench.py --trials --B 64 --max-steps 3000 --no-cpu \
    > $D/trials_small.json 2> $D/trials_small.err || { tail -30 $D/trials_small.err; exit 1; }
cat $D/trials_small.json
timeout -k 10 900 python -u scripts/episode_bench.py --trials --B ${TB:-4096} --assignment both \
    --cpu-budget 20 > $D/trials_c3.json 2> $D/trials_c3.err || { tail -30 $D/trials_c3.err; exit 1; }
cat $D/trials_c3.json
timeout -k 10 600 python -u scripts/episode_bench.py --assignment both --B 4096 --steps 3000 \
    > $D/episode_compare.json 2> $D/episode_compare.err || { tail -30 $D/episode_compare.err; exit 1; }
cat $D/episode_compare.json
