#!/bin/bash
# Per-dispatch kernel trace of one C5 batch (GEMM launch sizes and durations).
set -o pipefail
cd /root/repo
mkdir -p gpurun_out/c5trace
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace -d /tmp/c5t -o run --output-format csv -- python3 bench.py --config c5 --steps 1 --warmup 0 --no-cpu > gpurun_out/c5trace/log.txt 2>&1 || { echo "trace failed"; tail -20 gpurun_out/c5trace/log.txt; exit 1; }
f=$(find /tmp/c5t -name "*kernel_trace.csv" | head -1)
python3 - "$f" > gpurun_out/c5trace/dispatches.csv <<'PY'
import csv, sys
r = csv.DictReader(open(sys.argv[1]))
print("kernel,grid,start,end,dur_ns")
for d in r:
    k = d["Kernel_Name"]
    if "admm" in k or "gemm" in k:
        print('"%s",%s,%s,%s,%d' % (k.split("(")[0][:70], d.get("Grid_Size", d.get("Grid_Size_X", "")), d["Start_Timestamp"], d["End_Timestamp"], int(d["End_Timestamp"]) - int(d["Start_Timestamp"])))
PY
wc -l gpurun_out/c5trace/dispatches.csv
