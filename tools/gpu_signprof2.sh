# signing lines with the host-time profile (current build)
set -o pipefail
O=gpurun_out/signprof2
mkdir -p $O && export TMPDIR=/tmp
MPCX_HOST_PROFILE=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --extra-lines 0 --keygen-sessions 0 --no-cpu-baseline > $O/sign.json 2> $O/sign.err || { tail $O/sign.err; exit 1; }
python -c "
import json; d=json.load(open('$O/sign.json'))
for key in ('signing', 'signing_3_signers'):
    s=d[key]; print(key, round(s['value']), round(s['seconds'],3), 'busy', round(s['engine_busy_s'],3), 'host cpu', round(s['host_cpu_s'],2), {k: round(v,3) for k,v in s['rounds_s'].items()}); print('\n'.join(s.get('host_profile', [])[:24]))"
