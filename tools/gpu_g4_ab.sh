# One GPU call: parity suite after the 16x5 row_newbcast narrow geometry, then an
# A/B of the narrow-geometry threshold (mpcx_set_option narrow_rounds) on the
# signing and keygen lines.
set -o pipefail
mkdir -p gpurun_out/g4 && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/g4/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/g4/pytest_gpu.txt; [ $rc -eq 0 ] || exit 1
for nr in 15 15; do
  timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --extra-lines 0 --opt narrow_rounds=$nr > gpurun_out/g4/bench_nr$nr.json 2> gpurun_out/g4/bench_nr$nr.err || { tail gpurun_out/g4/bench_nr$nr.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/g4/bench_nr$nr.json').read().strip().splitlines()[-1]); print('narrow_rounds=$nr', round(d['value']), 'sign', round(d['signing']['value']), d['signing']['rounds_s'], 'keygen', round(d['keygen']['value'],1), round(d['keygen']['prove_s'],3), round(d['keygen']['verify_s'],3))"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/g4/sign -o sign -- python3 bench.py --count 1024 --steps 1 --warmup 1 --no-cpu-baseline --keygen-sessions 0 --extra-lines 0 > gpurun_out/g4/sign.json 2> gpurun_out/g4/sign.err || exit 1
timeout -k 10 200 python bench.py --count 1024 --steps 1 --warmup 1 --no-cpu-baseline --wallets 0 --keygen-sessions 0 > gpurun_out/g4/extra.json 2> gpurun_out/g4/extra.err || exit 1
python -c "import json; d=json.loads(open('gpurun_out/g4/extra.json').read().strip().splitlines()[-1]); print('paillier', round(d['paillier_batch']['value']), 'safe_prime', round(d['safe_prime']['value'],1))"
