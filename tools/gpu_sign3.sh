# signing parity, then chains vs round barriers on the signing lines
set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_signing.py tests/test_gpu_mta.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_sign.txt 2>&1 || { tail -30 gpurun_out/pytest_sign.txt; exit 1; }
tail -2 gpurun_out/pytest_sign.txt
for ch in 1 0 1 0; do
  MPCX_SIGN_CHAINS=$ch MPCX_HOST_PROFILE=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --extra-lines 0 --keygen-sessions 0 --no-cpu-baseline > gpurun_out/sign_ch$ch.json 2> gpurun_out/sign_ch$ch.err || { tail gpurun_out/sign_ch$ch.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/sign_ch$ch.json'))
for key in ('signing', 'signing_3_signers'):
    s=d[key]; idle=[l for l in s.get('host_profile',[]) if 'gpu_idle' in l]
    print('chains=$ch', key, round(s['value']), round(s['seconds'],3), round(s['engine_busy_s'],3), idle)"
done
