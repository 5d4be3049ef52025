# Host-time profile of the signing line, then kernel traces of the
# safe-prime/config-1 lines and of the signing line.
set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mta.py tests/test_gpu_wire.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_mta.txt 2>&1 || { tail -30 gpurun_out/pytest_mta.txt; exit 1; }
tail -3 gpurun_out/pytest_mta.txt
MPCX_HOST_PROFILE=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --extra-lines 0 --keygen-sessions 0 --no-cpu-baseline > gpurun_out/sign_hp.json 2> gpurun_out/sign_hp.err || { tail gpurun_out/sign_hp.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/sign_hp.json')); print(json.dumps(d.get('signing'), indent=0)[:3000])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sp_prof -o sp -- python3 bench.py --steps 1 --warmup 0 --wallets 0 --keygen-sessions 0 --no-cpu-baseline > gpurun_out/sp_prof.json 2> gpurun_out/sp_prof.err || { tail gpurun_out/sp_prof.err; exit 1; }
find gpurun_out/sp_prof -name '*kernel_stats*' -exec cut -c1-160 {} \;
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sign_prof -o sign -- python3 bench.py --steps 1 --warmup 0 --extra-lines 0 --keygen-sessions 0 --no-cpu-baseline > gpurun_out/sign_prof.json 2> gpurun_out/sign_prof.err || { tail gpurun_out/sign_prof.err; exit 1; }
find gpurun_out/sign_prof -name '*kernel_stats*' -exec cut -c1-160 {} \;
