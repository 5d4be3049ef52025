# signing lines with the host-time profile and process CPU time
set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_signing.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_sign.txt 2>&1 || { tail -30 gpurun_out/pytest_sign.txt; exit 1; }
tail -1 gpurun_out/pytest_sign.txt
for i in 1 2; do
MPCX_HOST_PROFILE=$((i % 2)) timeout -k 10 300 python bench.py --steps 1 --warmup 1 --extra-lines 0 --keygen-sessions 0 --no-cpu-baseline > gpurun_out/sign_hp$i.json 2> gpurun_out/sign_hp$i.err || { tail gpurun_out/sign_hp$i.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/sign_hp$i.json'))
for key in ('signing', 'signing_3_signers'):
    s=d[key]; print(key, round(s['value']), round(s['seconds'],3), 'busy', round(s['engine_busy_s'],3), 'host cpu', round(s['host_cpu_s'],2), s['rounds_s']); print('\n'.join(s.get('host_profile', [])))"
done
