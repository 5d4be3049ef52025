# kernel trace + host profile of the signing lines (2 and 3 signers)
set -o pipefail
O=gpurun_out/signtrace2
mkdir -p $O && export TMPDIR=/tmp
MPCX_HOST_PROFILE=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o sign -- python3 bench.py --steps 1 --warmup 1 --extra-lines 0 --keygen-sessions 0 --no-cpu-baseline > $O/sign.json 2> $O/sign.err || { tail $O/sign.err; exit 1; }
python -c "
import json; d=json.load(open('$O/sign.json'))
for key in ('signing', 'signing_3_signers'):
    s=d[key]; print(key, round(s['value']), round(s['seconds'],3), 'busy', round(s['engine_busy_s'],3), 'host cpu', round(s['host_cpu_s'],2), s['rounds_s']); print('\n'.join(s.get('host_profile', [])))"
