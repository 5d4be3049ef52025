#!/bin/bash
# Build tools/nat_asan.cpp against the host bignum with AddressSanitizer and
# UndefinedBehaviorSanitizer (host code only) and run it. CPU only.
set -e
cd "$(dirname "$0")/.."
out=${TMPDIR:-/tmp}/mpcx_nat_asan
H=mpcium_amd/csrc/host
g++ -O1 -g -std=c++17 -fsanitize=address,undefined -fno-sanitize-recover=undefined -I $H tools/nat_asan.cpp \
    $H/bignum.cpp $H/hostprof.cpp -lpthread -o $out
$out
