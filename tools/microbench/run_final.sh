# the round's last tree: GPU suite, smoke, the driver's default bench command
set -o pipefail
O=gpurun_out/r05/final3; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.txt 2>&1 || { tail -30 $O/suite.txt; exit 1; }
tail -2 $O/suite.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 900 python -u bench.py --detail $O/bench_detail.json > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
tail -c 2200 $O/bench.json
