# default bench line + kernel-trace stats of the same command into gpurun_out/$1
set -o pipefail
O=gpurun_out/${1:-benchprof}
mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench.json'))
print('config2', round(d['value']), d['roofline']['frac'], d['roofline']['kernel_ms'], d.get('batch_digest',{}).get('match'))
for s in d.get('config2_per_operand_exponents', []): print('  per-operand', s['exp_bits'], round(s['value']), s['kernel_ms'], round(s['roofline']['frac'],3))
for k in ('signing','signing_3_signers','keygen','safe_prime','paillier_batch'):
    s=d.get(k)
    if s: print(k, round(s['value'],1), s.get('unit'), (s.get('roofline') or {}).get('frac'), (s.get('cpu_baseline') or {}).get('value'))
"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --steps 3 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err || { tail $O/prof_bench.err; exit 1; }
find $O/prof -name '*kernel_stats*' -exec cut -c1-150 {} \; | head -14
