# fewer MtA launch phases (products as base^1 * mul after one exponentiation
# phase; WC EC check overlapped with the launches): MtA/signing GPU tests,
# then signing lines, new (build/ab_new) vs previous (build/ab_old) host library, interleaved
set -o pipefail
O=gpurun_out/phase_ab
mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_mta.py tests/test_gpu_signing.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pytest.txt | head -20; exit 1; }
for v in new old new old new old; do
  cp build/ab_$v/libmpcx_host.so mpcium_amd/libmpcx_host.so
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --extra-lines 0 --keygen-sessions 0 --no-cpu-baseline > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; cp build/ab_new/libmpcx_host.so mpcium_amd/; exit 1; }
  python -c "
import json; d=json.load(open('$O/ab.json'))
for key in ('signing', 'signing_3_signers'):
    s=d[key]; print('$v', key, round(s['value'],1), round(s['seconds'],3), 'busy', round(s['engine_busy_s'],3), {k: round(v, 3) for k, v in s['rounds_s'].items()})" | tee -a $O/ab.txt
done
cp build/ab_new/libmpcx_host.so mpcium_amd/libmpcx_host.so
