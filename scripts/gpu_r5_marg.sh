#!/bin/bash
# round 5: skip_margin (ABI 7) -- GPU tests of the touched paths, then the default bench
set -o pipefail
cd /root/repo
O=gpurun_out/r5_marg
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu \
    tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_gpu_facade.py \
    > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench.json'))
print(d['value'], d['ms_per_step'], d['margin'], d['stats'].get('fragile'), d['cpu_baseline']['value'])"
