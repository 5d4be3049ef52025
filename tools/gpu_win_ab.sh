# 5-bit fixed window for long per-operand exponents: modexp GPU tests, then the
# config-2 per-operand sub-lines and signing with fixed_window 5 vs 4, interleaved
set -o pipefail
O=gpurun_out/win_ab
mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_modexp.py tests/test_gpu_host.py tests/test_gpu_mta.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pytest.txt | head -20; exit 1; }
for w in 5 4 5 4; do
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --keygen-sessions 0 --no-cpu-baseline --opt fixed_window=$w > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/ab.json'))
print('win=$w config2', round(d['value']), [ (s['exp_bits'], round(s['value']), round(s['kernel_ms'],1), round(s['roofline']['frac'],3)) for s in d['config2_per_operand_exponents']], 'signing', round(d['signing']['value']), 'paillier', round(d['paillier_batch']['value']))" | tee -a $O/ab.txt
done
