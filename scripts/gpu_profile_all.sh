#!/bin/bash
# rocprofv3 kernel trace + stats of the bench, then the two PMC traffic passes.
set -o pipefail
cd /root/repo
bash scripts/gpu_prof.sh && bash scripts/gpu_pmc.sh
