#!/bin/bash
# Build the Engine (coalescers, pinned pool, comb-table cache) against the CPU
# mock of libmpcx (tools/mock_mpcx.cpp) with -fsanitize=address,undefined or
# -fsanitize=thread and run tools/engine_stress.cpp. CPU only, no GPU.
# usage: tools/engine_stress.sh [asan|tsan] [threads] [iters]
set -e
cd "$(dirname "$0")/.."
mode=${1:-asan}
threads=${2:-12}
iters=${3:-60}
H=mpcium_amd/csrc/host
case $mode in
  asan) san="-fsanitize=address,undefined -fno-omit-frame-pointer" ;;
  tsan) san="-fsanitize=thread" ;;
  *) echo "mode: asan or tsan" >&2; exit 2 ;;
esac
out=${TMPDIR:-/tmp}/mpcx_engine_stress_$mode
g++ -O1 -g -std=c++17 $san -pthread -I include -I $H tools/engine_stress.cpp tools/mock_mpcx.cpp \
    $H/engine.cpp $H/tsscommon.cpp $H/hostprof.cpp $H/bignum.cpp -lcrypto -o $out
MOCK_PIN_FAIL=${MOCK_PIN_FAIL:-100} ASAN_OPTIONS=detect_leaks=0 TSAN_OPTIONS=halt_on_error=1 $out $threads $iters
