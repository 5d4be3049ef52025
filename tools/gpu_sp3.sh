# prime-path parity (cooperative and thread-per-candidate kernels), then the
# config-3 line A/B and its kernel trace
set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_primes.py tests/test_gpu_host.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_sp.txt 2>&1 || { tail -40 gpurun_out/pytest_sp.txt; exit 1; }
tail -3 gpurun_out/pytest_sp.txt
for c in 1 0; do
  timeout -k 10 300 python bench.py --steps 1 --warmup 0 --count 4096 --wallets 0 --keygen-sessions 0 --no-cpu-baseline --opt prime_coop=$c > gpurun_out/sp_bench_$c.json 2> gpurun_out/sp_bench_$c.err || { tail gpurun_out/sp_bench_$c.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/sp_bench_$c.json'))['safe_prime']; print('coop=$c', round(d['value'],1), 'primes/s', round(d['fermat_tests_per_s']/1e6,3), 'M tests/s', d['seconds'], d['mr_tests'], d['lucas_tests'], round(d['roofline']['frac'],3))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sp_prof3 -o sp -- python3 bench.py --steps 1 --warmup 0 --count 4096 --wallets 0 --keygen-sessions 0 --no-cpu-baseline > gpurun_out/sp_prof3.json 2> gpurun_out/sp_prof3.err || { tail gpurun_out/sp_prof3.err; exit 1; }
find gpurun_out/sp_prof3 -name '*kernel_stats*' -exec cut -c1-150 {} \;
