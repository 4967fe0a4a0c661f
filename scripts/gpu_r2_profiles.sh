#!/bin/bash
# Round-2 evidence for one bench config (CFG=c3|c4|c2): the bench line, the
# rocprofv3 kernel-trace summary of the same command, the HBM traffic PMC
# passes and the auction kernel's SQ counter passes. Everything lands in
# gpurun_out/r2_$CFG; scripts/pmc_*summary.py turn it into profiles/.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
CFG=${CFG:-c3}
O=gpurun_out/r2_$CFG
mkdir -p $O
case $CFG in
  c3) AARGS="--B 65536 --n 100" ;;
  c4) AARGS="--B 2048 --n 500 --L 90" ;;
  c2) AARGS="--B 4096 --n 20 --L 15 --complete"; GRAPH=--graph ;;  # launch-bound: graph replay
esac
[ -n "$SKIP_BENCH" ] || timeout -k 10 600 python3 bench.py --config $CFG $GRAPH > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
rm -rf /tmp/kt_$CFG
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/kt_$CFG -o run --output-format csv -- \
    python3 bench.py --config $CFG --steps 5 --warmup 2 --no-cpu --no-ca-probe > $O/bench_kt.json 2> $O/kt.err || { echo "kernel trace failed"; tail -20 $O/kt.err; exit 1; }
f=$(find /tmp/kt_$CFG -name "*kernel_stats.csv" | head -1)
cp "$f" $O/kernel_stats.csv
mkdir -p $O/pmc
for C in FETCH_SIZE WRITE_SIZE; do
  rm -rf /tmp/pmc_$C
  timeout -k 10 -s KILL 600 rocprofv3 --pmc $C -d /tmp/pmc_$C -o run --output-format csv -- \
      python3 bench.py --config $CFG --steps 2 --warmup 1 --no-cpu --no-setup-ab --no-ca-probe \
      > $O/pmc/bench_$C.json 2> $O/pmc/rocprof_$C.err || { echo "pmc $C failed"; tail -20 $O/pmc/rocprof_$C.err; exit 1; }
  f=$(find /tmp/pmc_$C -name "*counter_collection.csv" | head -1)
  head -1 "$f" > $O/pmc/$C.csv
  grep "acl_amd" "$f" >> $O/pmc/$C.csv
done
[ -n "$SKIP_SQ" ] || OUT=r2_$CFG/pmca AUCTION_ARGS="$AARGS" bash scripts/gpu_pmc_auction.sh
