#!/bin/bash
# Build an experiment variant of the library: scripts/build_variant.sh NAME [SRCDIR] [extra hipcc flags]
# -> aclswarm_amd/lib/exp/NAME.so (load it with ACLSWARM_AMD_LIB=...). SRCDIR defaults to
# aclswarm_amd/csrc (e.g. a `git archive` of another commit's csrc for a same-box A/B).
set -e
cd "$(dirname "$0")/.."
name=$1; shift
C=aclswarm_amd/csrc
if [ $# -gt 0 ] && [ -d "$1" ]; then C=$1; shift; fi
mkdir -p aclswarm_amd/lib/exp
SRCS=$(python3 -c "from aclswarm_amd import build; print(' '.join(build.SOURCES))")
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -shared -Wall -Wno-unused-function "$@" \
  $(for f in $SRCS; do echo $C/$f; done) -o aclswarm_amd/lib/exp/$name.so
