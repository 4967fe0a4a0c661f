#!/bin/bash
# Round-5 phase study of the C3 fused kernel: bench line, stamp phase split
# (fused control share), PROF-build CBAA sections, per-phase SQ instruction
# counts (stop builds, fused path). Outputs under gpurun_out/$OUT.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=${OUT:-r5_phase}
mkdir -p gpurun_out/$OUT
timeout -k 10 300 python bench.py > gpurun_out/$OUT/bench.json 2> gpurun_out/$OUT/bench.err || { tail -20 gpurun_out/$OUT/bench.err; exit 1; }
tail -c 600 gpurun_out/$OUT/bench.json
timeout -k 10 200 python scripts/phase_profile.py > gpurun_out/$OUT/phase.txt 2>&1 || { tail -20 gpurun_out/$OUT/phase.txt; exit 1; }
cat gpurun_out/$OUT/phase.txt
ACLSWARM_AMD_LIB=$PWD/aclswarm_amd/lib/exp/prof.so timeout -k 10 200 python scripts/phase_profile.py --no-control > gpurun_out/$OUT/phase_prof.txt 2>&1 || { tail -20 gpurun_out/$OUT/phase_prof.txt; exit 1; }
cat gpurun_out/$OUT/phase_prof.txt
[ -n "$NO_PMC" ] && exit 0
OUT=$OUT/pmc AO_ARGS="--control --B 65536" STOPS="${STOPS:-1 2 3 4 5 0}" bash scripts/auction_phase_pmc.sh
