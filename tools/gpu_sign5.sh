# MtA + signing GPU tests, then signing A/B: paired entries (halves concurrent,
# one range-proof verification) vs separate BobMid / BobMidWC calls, interleaved
set -o pipefail
O=gpurun_out/sign5
mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_mta.py tests/test_gpu_signing.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; tail -3 $O/pytest.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pytest.txt | head -20; exit 1; }
for pr in 1 0 1 0 1 0; do
  MPCX_SIGN_PAIRED=$pr timeout -k 10 300 python bench.py --steps 1 --warmup 1 --extra-lines 0 --keygen-sessions 0 --no-cpu-baseline > $O/sign_ab.json 2> $O/sign_ab.err || { tail $O/sign_ab.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/sign_ab.json'))
for key in ('signing', 'signing_3_signers'):
    s=d[key]; print('paired=$pr', key, round(s['value']), round(s['seconds'],3), 'busy', round(s['engine_busy_s'],3), 'cpu', round(s['host_cpu_s'],1))" | tee -a $O/sign_ab.txt
done
