#!/bin/bash
# Object-level builds for kernel experiments: compiles every source once into
# build/obj/, then links variants with auction.hip rebuilt under extra flags:
#   scripts/build_objs.sh VARIANT [hipcc flags for auction.hip ...]
# -> aclswarm_amd/lib/exp/VARIANT.so (load with ACLSWARM_AMD_LIB=...)
set -e
cd "$(dirname "$0")/.."
C=aclswarm_amd/csrc
F="-O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -Wall -Wno-unused-function"
mkdir -p build/obj aclswarm_amd/lib/exp
for s in solve solve_wide control admm hungarian episode trial formation_gen; do
  o=build/obj/$s.o
  if [ ! -f $o ] || [ $C/$s.hip -nt $o ] || [ $C/common.h -nt $o ] || [ $C/control_params.h -nt $o ] || [ $C/umeyama_dev.h -nt $o ] || [ include/aclswarm_amd.h -nt $o ]; then
    /opt/rocm/bin/hipcc $F -c $C/$s.hip -o $o
  fi
done
{ [ build/obj/api.o -nt $C/api.cpp ] && [ build/obj/api.o -nt include/aclswarm_amd.h ]; } || /opt/rocm/bin/hipcc $F -c $C/api.cpp -o build/obj/api.o
name=$1; shift
/opt/rocm/bin/hipcc $F "$@" -c $C/auction.hip -o build/obj/auction_$name.o
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 build/obj/{solve,solve_wide,control,admm,hungarian,episode,trial,formation_gen,api}.o build/obj/auction_$name.o -o aclswarm_amd/lib/exp/$name.so
echo aclswarm_amd/lib/exp/$name.so
