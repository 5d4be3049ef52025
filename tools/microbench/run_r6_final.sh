# the driver's default bench on the current tree, then the same command under
# rocprofv3 --kernel-trace --stats (per-kernel durations for the roofline cross-check)
set -o pipefail
O=gpurun_out/r06/$1; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py --detail $O/bench_detail.json > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
wc -c $O/bench.json
python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print(d['value'], r['frac'], r.get('go_equiv_frac'), r['kernel_ms'], {k: v['value'] for k, v in d.get('configs', {}).items()})"
timeout -k 10 560 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --steps 5 --warmup 1 --wallets 0 --keygen-sessions 0 --extra-lines 0 --no-cpu-baseline --detail $O/trace_bench_detail.json > $O/trace_bench.json 2> $O/trace_bench.err || { tail $O/trace_bench.err; exit 1; }
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 tools/trace_segments.py $f > $O/trace_segments.txt && head -20 $O/trace_segments.txt
find $O/prof -name '*kernel_stats*' -exec cp {} $O/kernel_stats.csv \;
