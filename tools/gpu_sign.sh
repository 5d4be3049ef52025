# MtA / signing / proof parity on the GPU, then the signing lines with the
# host-time profile.
set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mta.py tests/test_gpu_wire.py tests/test_gpu_signing.py tests/test_gpu_proofs.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_sign.txt 2>&1 || { tail -30 gpurun_out/pytest_sign.txt; exit 1; }
tail -2 gpurun_out/pytest_sign.txt
MPCX_HOST_PROFILE=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --extra-lines 0 --keygen-sessions 0 --no-cpu-baseline > gpurun_out/sign_hp.json 2> gpurun_out/sign_hp.err || { tail gpurun_out/sign_hp.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/sign_hp.json'))
for key in ('signing', 'signing_3_signers'):
    s=d[key]; [s.pop(k, None) for k in ('metric','scope','checked','roofline')]; print(key, json.dumps(s, indent=0)[:2500])"
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --extra-lines 0 --keygen-sessions 0 --no-cpu-baseline > gpurun_out/sign_np.json 2> gpurun_out/sign_np.err || { tail gpurun_out/sign_np.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/sign_np.json'))
for key in ('signing', 'signing_3_signers'): s=d[key]; print(key, round(s['value']), s['seconds'], s['engine_busy_s'], round(s['host_share'],3), s['roofline']['frac'])"
