# libmpcx.so A/B (build/ab/libmpcx_new.so vs build/ab/libmpcx_base.so): GPU tests
# on the new build, then interleaved bench lines given as arguments to bench.py
set -o pipefail
O=gpurun_out/lib_ab
mkdir -p $O && export TMPDIR=/tmp
cp build/ab/libmpcx_new.so mpcium_amd/libmpcx.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_primes.py tests/test_gpu_host.py tests/test_gpu_modexp.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pytest.txt | head -20; exit 1; }
for v in new base new base new base; do
  cp build/ab/libmpcx_$v.so mpcium_amd/libmpcx.so
  timeout -k 10 300 python bench.py "$@" > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; cp build/ab/libmpcx_new.so mpcium_amd/libmpcx.so; exit 1; }
  python -c "
import json; d=json.load(open('$O/ab.json'))
out=['$v', 'config2', round(d['value'])]
for k in ('safe_prime', 'keygen', 'signing', 'paillier_batch'):
    if k in d: out += [k, round(d[k]['value'], 1)]
print(*out)" | tee -a $O/ab.txt
done
cp build/ab/libmpcx_new.so mpcium_amd/libmpcx.so
