#!/bin/bash
# Build the host worker pool with -fsanitize=thread (host code only) and run
# tools/pool_stress.cpp: nested parallel loops from many threads. CPU only.
set -e
cd "$(dirname "$0")/.."
out=${TMPDIR:-/tmp}/mpcx_pool_tsan
H=mpcium_amd/csrc/host
g++ -O1 -g -std=c++17 -fsanitize=thread -pthread -I include -I $H tools/pool_stress.cpp $H/tsscommon.cpp \
    $H/hostprof.cpp $H/bignum.cpp -L mpcium_amd -lmpcx -lcrypto -Wl,-rpath,$PWD/mpcium_amd -o $out
$out
