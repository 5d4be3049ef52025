# Full validation of the current build: GPU suite, smoke, default bench line,
# kernel trace of the bench command.
set -o pipefail
mkdir -p gpurun_out/full3 && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/full3/pytest_gpu.txt 2>&1
rc=$?; tail -3 gpurun_out/full3/pytest_gpu.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/full3/pytest_gpu.txt | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full3/smoke.txt 2>&1 || { tail gpurun_out/full3/smoke.txt; exit 1; }
tail -2 gpurun_out/full3/smoke.txt
timeout -k 10 900 python bench.py > gpurun_out/full3/bench.json 2> gpurun_out/full3/bench.err || { tail gpurun_out/full3/bench.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/full3/bench.json'))
print('config2', round(d['value']), d['roofline']['frac'], d['roofline']['kernel_ms'], d.get('batch_digest',{}).get('match'))
for s in d.get('config2_per_operand_exponents', []): print('  per-operand', s['exp_bits'], round(s['value']), s['kernel_ms'], round(s['roofline']['frac'],3))
for k in ('signing','signing_3_signers','keygen','safe_prime','paillier_batch'):
    s=d.get(k); 
    if s: print(k, round(s['value'],1), s.get('unit'), (s.get('roofline') or {}).get('frac'), (s.get('cpu_baseline') or {}).get('value'))
print('cpu', json.dumps(d.get('cpu_baseline'))[:400])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/full3/prof -o bench -- python3 bench.py --steps 3 --no-cpu-baseline > gpurun_out/full3/prof_bench.json 2> gpurun_out/full3/prof_bench.err || { tail gpurun_out/full3/prof_bench.err; exit 1; }
find gpurun_out/full3/prof -name '*kernel_stats*' -exec cut -c1-150 {} \;
