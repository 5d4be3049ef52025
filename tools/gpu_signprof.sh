# signing lines with the host-time profile only
set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
MPCX_HOST_PROFILE=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --extra-lines 0 --keygen-sessions 0 --no-cpu-baseline > gpurun_out/sign_hp.json 2> gpurun_out/sign_hp.err || { tail gpurun_out/sign_hp.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/sign_hp.json'))
for key in ('signing', 'signing_3_signers'):
    s=d[key]; print(key, round(s['value']), s['seconds'], s['engine_busy_s'], s['rounds_s']); print('\n'.join(s['host_profile']))"
