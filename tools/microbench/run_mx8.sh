# k_modexp_multi_mx: parity tests, then signing / config-1 lines with and without it (interleaved, 2 rounds)
set -o pipefail
O=gpurun_out/mx8; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_mx.py -x -q --timeout 380 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for r in 1 2; do for v in on off; do
  if [ $v = on ]; then X=""; else X="--opt mx_seg_min=100000000"; fi
  timeout -k 10 500 python -u bench.py --steps 2 --warmup 1 --keygen-sessions 0 --no-cpu-baseline $X --detail $O/d_${v}_$r.json > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail $O/b_${v}_$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/b_${v}_$r.json').read().strip().splitlines()[-1]); c=d['configs']
print('$v $r', d['value'], c['c4_sign']['value'], c['c4_sign_3_signers']['value'], c['c1_paillier']['value'], c['c1_paillier'].get('in_flight_value'))"
done; done
