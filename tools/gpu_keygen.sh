# keygen/reshare proof driver: parity tests, then the config-5 line twice
set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_proofs.py tests/test_gpu_signing.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_kg.txt 2>&1 || { tail -30 gpurun_out/pytest_kg.txt; exit 1; }
tail -1 gpurun_out/pytest_kg.txt
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --wallets 0 --extra-lines 0 --no-cpu-baseline > gpurun_out/kg$i.json 2> gpurun_out/kg$i.err || { tail gpurun_out/kg$i.err; exit 1; }
  python -c "
import json; s=json.load(open('gpurun_out/kg$i.json'))['keygen']; print('keygen', round(s['value'],1), s['seconds'], s.get('engine_busy_s'), s.get('prove_s'), s.get('verify_s'), s['roofline']['frac'])"
done
