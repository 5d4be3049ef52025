#!/bin/bash
# Build libmpcx_host.so from the host sources of git revision REV (for an
# interleaved A/B of host-side protocol changes: tools/gpu.sh abhost), linked
# against the current libmpcx.so (same C-ABI). usage: tools/build_host_variant.sh REV OUT_DIR
set -e
cd "$(dirname "$0")/.."
rev=$1; out=$2
mkdir -p $out/src
git archive $rev mpcium_amd/csrc/host include | tar -x -C $out/src
H=$out/src/mpcium_amd/csrc/host
objs=()
for f in $H/*.cpp; do
  o=$out/$(basename ${f%.cpp}).o
  g++ -O3 -std=c++17 -fPIC -Wall -pthread -I $out/src/include -I $H -c -o $o $f &
  objs+=($o)
done
wait
g++ -shared -pthread -o $out/libmpcx_host.so ${objs[@]} -L mpcium_amd -lmpcx -lcrypto -Wl,-rpath,'$ORIGIN'
echo $out/libmpcx_host.so
