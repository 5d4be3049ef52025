# config-3 step size at the bench's 64 primes (3 interleaved runs)
set -o pipefail
for i in 1 2 3; do
  for b in 524288 655360 786432; do
    echo -n "batch=$b: "
    MPCX_SAFEPRIME_BATCH=$b timeout -k 10 120 python tools/sp_prof.py 64 8 | head -1 | cut -c1-60 || exit 1
  done
done
