# config 3: cooperative (k_prime2c / k_mrc) vs thread-per-candidate prime kernels at the 2^19 step, interleaved
set -o pipefail
O=gpurun_out/sp_ab
mkdir -p $O && export TMPDIR=/tmp
for pc in 1 0 1 0 1 0; do
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --wallets 0 --keygen-sessions 0 --no-cpu-baseline --opt prime_coop=$pc > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/ab.json'))
s=d['safe_prime']; print('prime_coop=$pc', round(s['value'],1), 'fermat/s', round(s['fermat_tests_per_s']), round(s['seconds'],4))" | tee -a $O/ab.txt
done
