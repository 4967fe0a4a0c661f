#!/bin/bash
# acl_tile_gains: parity tests, timing, and its HBM traffic (two PMC passes)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/tile
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "tiled or directed" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python3 scripts/tile_only.py || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
  rm -rf /tmp/tpmc_$C
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $C -d /tmp/tpmc_$C -o run --output-format csv -- python3 scripts/tile_only.py --reps 1 > $O/out_$C.txt 2> $O/err_$C.txt || { echo "pmc $C failed"; tail -20 $O/err_$C.txt; exit 1; }
  f=$(find /tmp/tpmc_$C -name "*counter_collection.csv" | head -1)
  head -1 "$f" > $O/$C.csv
  grep tile_gains "$f" >> $O/$C.csv
done
python3 - <<'PY'
import csv
v = {}
for C in ("FETCH_SIZE", "WRITE_SIZE"):
    r = list(csv.DictReader(open("gpurun_out/tile/%s.csv" % C)))
    v[C] = sum(float(x["Counter_Value"]) for x in r) / len(r) * 1024.0
print("tile_gains per launch: FETCH_SIZE %.2f GB (x2 = %.2f GB), WRITE_SIZE %.2f GB, hbm %.2f GB" % (
    v["FETCH_SIZE"] / 1e9, 2 * v["FETCH_SIZE"] / 1e9, v["WRITE_SIZE"] / 1e9,
    (2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) / 1e9))
PY
