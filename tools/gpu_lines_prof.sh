# One GPU call: kernel-trace profiles of the signing (config 4) and keygen
# (config 5) lines separately, to see which kernels and geometries carry them.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/lines
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/sign -o sign -- python3 bench.py --count 1024 --steps 1 --warmup 1 --no-cpu-baseline --keygen-sessions 0 --extra-lines 0 > $OUT/sign.json 2> $OUT/sign.err || { tail $OUT/sign.err; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/keygen -o keygen -- python3 bench.py --count 1024 --steps 1 --warmup 1 --no-cpu-baseline --wallets 0 --extra-lines 0 > $OUT/keygen.json 2> $OUT/keygen.err || { tail $OUT/keygen.err; exit 1; }
for f in sign keygen; do echo "== $f"; find $OUT/$f -name '*kernel_stats*' -exec cut -d, -f1-4 {} \; | head -12; done
