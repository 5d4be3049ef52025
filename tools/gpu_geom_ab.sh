# mid geometry + launch-time model: modexp GPU tests, then signing / keygen
# lines with MPCX_GEOM_POLICY=1 (model) vs 0 (round-1 thresholds), interleaved
set -o pipefail
O=gpurun_out/geom_ab
mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_modexp.py tests/test_gpu_host.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pytest.txt | head -20; exit 1; }
for gp in 1 0 1 0; do
  MPCX_GEOM_POLICY=$gp timeout -k 10 300 python bench.py --steps 1 --warmup 1 --extra-lines 0 --no-cpu-baseline > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/ab.json'))
print('policy=$gp config2', round(d['value']))
for key in ('signing', 'signing_3_signers', 'keygen'):
    s=d[key]; print('policy=$gp', key, round(s['value'],1), round(s['seconds'],3), 'busy', round(s['engine_busy_s'],3))" | tee -a $O/ab.txt
done
