# interleaved config-2 timing of two libmpcx builds (timing-only variants)
set -o pipefail
for i in 1 2 3; do
  for l in mpcium_amd/libmpcx.so build/ab/libmpcx_nomul.so; do
    timeout -k 10 120 python tools/ab_time.py $l 4 || exit 1
  done
done
