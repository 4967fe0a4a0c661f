set -o pipefail
cd /root/repo
mkdir -p gpurun_out/crowd
for a in "--B 65536 --n 100" "--B 65536 --n 100 --crowd 0.3" "--B 2048 --n 500 --L 90" "--B 2048 --n 500 --L 90 --crowd 0.3"; do
  timeout -k 10 200 python3 scripts/auction_only.py --control --hist --reps 3 $a >> gpurun_out/crowd/out.txt 2>&1 || { tail -20 gpurun_out/crowd/out.txt; exit 1; }
done
cat gpurun_out/crowd/out.txt
OUT=r4_c4_sqa AUCTION_ARGS="--B 2048 --n 500 --L 90 --control" bash scripts/gpu_pmc_auction.sh > gpurun_out/sqa.txt 2>&1 || { tail -20 gpurun_out/sqa.txt; exit 1; }
grep align gpurun_out/sqa.txt
