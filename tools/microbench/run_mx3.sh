# full GPU suite and the default bench with k_modexp_mx on by default
set -o pipefail
O=gpurun_out/mx3; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.txt 2>&1 || { tail -30 $O/suite.txt; exit 1; }
tail -2 $O/suite.txt
timeout -k 10 900 python -u bench.py --detail $O/bench_detail.json > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 tools/ab_summary.py $O $O/summary.json "default bench, mx on" 2>/dev/null; tail -c 1500 $O/bench.json
