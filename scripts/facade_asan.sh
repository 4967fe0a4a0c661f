#!/bin/bash
# Host AddressSanitizer + UndefinedBehaviorSanitizer over the facade's
# exchange-mode protocol (tests/exchange_asan_main.cpp), linked to the
# in-tree libaclswarm_amd.so (its GPU code is not instrumented). Run on the
# GPU box: bash scripts/facade_asan.sh  (writes gpurun_out/${OUT:-facade_asan}/)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${OUT:-facade_asan}
mkdir -p $O
g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -Wall -Wextra -Werror \
    -Iinclude tests/exchange_asan_main.cpp -Laclswarm_amd/lib -laclswarm_amd \
    -Wl,-rpath,$PWD/aclswarm_amd/lib -o $O/exchange_asan || exit 1
ASAN_OPTIONS=detect_leaks=0:abort_on_error=0:halt_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
    timeout -k 10 300 $O/exchange_asan > $O/exchange_asan.txt 2>&1
e=$?
tail -20 $O/exchange_asan.txt
exit $e
