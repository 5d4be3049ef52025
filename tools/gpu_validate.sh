# One GPU call: parity tests, smoke, default bench line, kernel-trace profile of the bench.
set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || { cat gpurun_out/smoke.txt; exit 1; }
tail -1 gpurun_out/smoke.txt
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --wallets 0 > gpurun_out/prof_bench.json 2>gpurun_out/prof.err || { tail gpurun_out/prof.err; exit 1; }
cat gpurun_out/prof_bench.json
find gpurun_out/prof -name '*kernel_stats*' -exec cat {} \;
