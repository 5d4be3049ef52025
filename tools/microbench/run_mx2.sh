# MX kernel: microbench check + timing, GPU parity tests, config-2 bench with and without MX
set -o pipefail
O=gpurun_out/mx2; mkdir -p $O
(cd tools/microbench && timeout -k 10 100 python -u mx_chain.py 16 1 debug > ../../$O/dbg.json 2> ../../$O/dbg.err && timeout -k 10 150 python -u mx_chain.py 65536 64 > ../../$O/chain.json 2>> ../../$O/dbg.err) || { cat $O/dbg.err | tail; exit 1; }
cat $O/dbg.json $O/chain.json
timeout -k 10 300 python -u -m pytest tests/test_gpu_mx.py -x -q --timeout 280 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for mx in 1 0; do timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --extra-lines 0 --wallets 0 --keygen-sessions 0 --no-cpu-baseline --opt mx=$mx --detail $O/detail_mx$mx.json > $O/bench_mx$mx.json 2> $O/bench_mx$mx.err || { tail $O/bench_mx$mx.err; exit 1; }; python3 -c "
import json; d=json.loads(open('$O/bench_mx$mx.json').read().strip().splitlines()[-1]); print('mx=$mx', d['value'], d['ms_per_step'], d['roofline']['frac'])"; done
