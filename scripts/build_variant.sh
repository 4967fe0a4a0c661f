#!/bin/bash
# Build an experiment variant of the library: scripts/build_variant.sh NAME [extra hipcc flags]
# -> aclswarm_amd/lib/exp/NAME.so (load it with ACLSWARM_AMD_LIB=...)
set -e
cd "$(dirname "$0")/.."
name=$1; shift
C=aclswarm_amd/csrc
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -shared -Wall -Wno-unused-function "$@" \
  $C/solve.hip $C/solve_wide.hip $C/control.hip $C/admm.hip $C/hungarian.hip $C/episode.hip $C/formation_gen.hip $C/api.cpp -o aclswarm_amd/lib/exp/$name.so
