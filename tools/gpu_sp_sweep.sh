# config-3 step size x prime-kernel layout sweep (256 safe primes: steady state)
set -o pipefail
for pc in 1 0; do
  for b in 458752 524288 786432 917504 1048576; do
    echo -n "coop=$pc batch=$b: "
    MPCX_SAFEPRIME_BATCH=$b MPCX_PRIME_COOP=$pc timeout -k 10 120 python tools/sp_prof.py 256 8 | head -1 || exit 1
  done
done
