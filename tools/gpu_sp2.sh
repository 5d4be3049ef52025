# GPU suite, then the config-3 (safe-prime) line alone plus its kernel trace.
set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_gpu.txt | tail -25; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --wallets 0 --keygen-sessions 0 --no-cpu-baseline > gpurun_out/sp_bench.json 2> gpurun_out/sp_bench.err || { tail gpurun_out/sp_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/sp_bench.json')); print(json.dumps(d['safe_prime']))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sp_prof -o sp -- python3 bench.py --steps 1 --warmup 0 --wallets 0 --keygen-sessions 0 --no-cpu-baseline > gpurun_out/sp_prof.json 2> gpurun_out/sp_prof.err || { tail gpurun_out/sp_prof.err; exit 1; }
find gpurun_out/sp_prof -name '*kernel_stats*' -exec cat {} \;
