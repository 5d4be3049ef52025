# Full validation of the current build: GPU suite, smoke, signing paired-batch
# A/B (interleaved), default bench line, kernel trace of the bench command.
set -o pipefail
O=gpurun_out/full3
mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -3 $O/pytest_gpu.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pytest_gpu.txt | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
for pr in 1 0 1 0; do
  MPCX_SIGN_PAIRED=$pr timeout -k 10 300 python bench.py --steps 1 --warmup 1 --extra-lines 0 --keygen-sessions 0 --no-cpu-baseline > $O/sign_ab.json 2> $O/sign_ab.err || { tail $O/sign_ab.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/sign_ab.json'))
for key in ('signing', 'signing_3_signers'):
    s=d[key]; print('paired=$pr', key, round(s['value']), round(s['seconds'],3), 'busy', round(s['engine_busy_s'],3), 'cpu', round(s['host_cpu_s'],1))" | tee -a $O/sign_ab.txt
done
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench.json'))
print('config2', round(d['value']), d['roofline']['frac'], d['roofline']['kernel_ms'], d.get('batch_digest',{}).get('match'))
for s in d.get('config2_per_operand_exponents', []): print('  per-operand', s['exp_bits'], round(s['value']), s['kernel_ms'], round(s['roofline']['frac'],3))
for k in ('signing','signing_3_signers','keygen','safe_prime','paillier_batch'):
    s=d.get(k)
    if s: print(k, round(s['value'],1), s.get('unit'), (s.get('roofline') or {}).get('frac'), (s.get('cpu_baseline') or {}).get('value'))
"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --steps 3 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err || { tail $O/prof_bench.err; exit 1; }
find $O/prof -name '*kernel_stats*' -exec cut -c1-150 {} \;
