#!/bin/bash
# run the C2/C1 parity tests against library variants: scripts/gpu_bisect.sh V ...
cd /root/repo
for v in "$@"; do echo "== $v"; ACLSWARM_AMD_LIB=$PWD/aclswarm_amd/lib/exp/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 -k "c2_full or c2 or swarm6" 2>&1 | tail -2; done
