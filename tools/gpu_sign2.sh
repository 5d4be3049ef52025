# signing parity, then a sweep of the chunk-pipeline setting on the signing line
set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_signing.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_sign.txt 2>&1 || { tail -30 gpurun_out/pytest_sign.txt; exit 1; }
tail -2 gpurun_out/pytest_sign.txt
for pl in 1,1 4,2 8,2 8,3 6,3 8,4; do
  MPCX_SIGN_PIPELINE=$pl timeout -k 10 300 python bench.py --steps 1 --warmup 1 --extra-lines 0 --keygen-sessions 0 --no-cpu-baseline > gpurun_out/sign_$pl.json 2> gpurun_out/sign_$pl.err || { tail gpurun_out/sign_$pl.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/sign_$pl.json')); s=d['signing']; t=d.get('signing_3_signers',{}); print('$pl', round(s['value']), round(s['host_share'],3), s['engine_busy_s'], s['seconds'], s['rounds_s'], '| 3 signers', round(t.get('value',0)))"
done
