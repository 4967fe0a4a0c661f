#!/bin/bash
# HBM traffic of the bench's kernels from PMC counters: two separate
# rocprofv3 passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950,
# MI355X_MICROARCH.md "rocprofv3 PMC slots"), counters only -- no traces.
set -o pipefail
cd /root/repo
OUT=${OUT:-pmc}
export TMPDIR=/tmp
mkdir -p gpurun_out/$OUT
for C in FETCH_SIZE WRITE_SIZE; do
  rm -rf /tmp/pmc_$C
  timeout -k 10 600 rocprofv3 --pmc $C -d /tmp/pmc_$C -o run --output-format csv -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu --no-ca-probe ${BENCH_ARGS} \
      > gpurun_out/$OUT/bench_$C.json 2> gpurun_out/$OUT/rocprof_$C.err || { echo "pmc $C failed"; tail -20 gpurun_out/$OUT/rocprof_$C.err; exit 1; }
  f=$(find /tmp/pmc_$C -name "*counter_collection.csv" | head -1)
  head -1 "$f" > gpurun_out/$OUT/$C.csv
  grep "acl_amd" "$f" >> gpurun_out/$OUT/$C.csv
done
wc -l gpurun_out/$OUT/*.csv
