#!/bin/bash
# Tiled gain records: GPU parity tests, then the bench with and without the
# tile-ordered copy.
set -o pipefail
mkdir -p gpurun_out
cd /root/repo
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_tiled.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_tiled.log; exit 1; }
grep -cE "PASSED" gpurun_out/pytest_tiled.log; tail -2 gpurun_out/pytest_tiled.log
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_tiled.json 2> gpurun_out/bench_tiled.err || { echo "bench failed"; tail -30 gpurun_out/bench_tiled.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu --no-tile-gains > gpurun_out/bench_rows.json 2> gpurun_out/bench_rows.err || { echo "bench failed"; tail -30 gpurun_out/bench_rows.err; exit 1; }
python - <<'PY'
import json
for f in ("bench_tiled", "bench_rows"):
    d = json.load(open(f"gpurun_out/{f}.json"))
    k = d["roofline"]["kernels"]
    print(f, round(d["value"]), round(d["ms_per_step"], 3), {n: round(v["avg_launch_ms"], 3) for n, v in k.items()}, round(d["roofline"]["frac"], 4), d["config"]["gain_layout"])
PY
