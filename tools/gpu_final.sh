# One GPU call: FETCH_SIZE / WRITE_SIZE passes of the current bench kernel
# (installed as the bench's traffic source on the box), then the default bench
# line and a kernel-trace profile of the config-2 kernel alone.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/final
bash tools/gpu_pmc_traffic.sh > gpurun_out/final/pmc.txt 2>&1 || { cat gpurun_out/final/pmc.txt; exit 1; }
cat gpurun_out/final/pmc.txt
cp gpurun_out/pmc/summary.json profiles/r01/pmc_traffic/summary.json
timeout -k 10 400 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || { tail gpurun_out/final/bench.err; exit 1; }
cat gpurun_out/final/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/prof -o bench -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --wallets 0 --keygen-sessions 0 --extra-lines 0 > gpurun_out/final/prof_bench.json 2> gpurun_out/final/prof.err || { tail gpurun_out/final/prof.err; exit 1; }
cat gpurun_out/final/prof_bench.json
find gpurun_out/final/prof -name '*kernel_stats*' -exec cat {} \;
