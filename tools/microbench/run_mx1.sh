set -o pipefail
mkdir -p gpurun_out/mxt
cd tools/microbench
for v in t1 t2; do MX_CHAIN_SO=mx_chain_$v.so timeout -k 10 120 python -u mx_chain.py 65536 64 > ../../gpurun_out/mxt/chain_$v.json 2>/dev/null || exit 1; done
timeout -k 10 120 python -u mx_chain.py 65536 64 > ../../gpurun_out/mxt/chain_full.json 2>/dev/null || exit 1
cd ../..
for mx in 1 0; do timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --extra-lines 0 --wallets 0 --keygen-sessions 0 --no-cpu-baseline --opt mx=$mx --detail gpurun_out/mxt/detail_mx$mx.json > gpurun_out/mxt/bench_mx$mx.json 2> gpurun_out/mxt/bench_mx$mx.err || exit 1; done
cat gpurun_out/mxt/chain_*.json; for mx in 1 0; do python -c "
import json; d=json.loads(open('gpurun_out/mxt/bench_mx$mx.json').read().strip().splitlines()[-1]); print($mx, d['value'], d['ms_per_step'], d['roofline']['frac'], [ (x.get('value'),x.get('frac')) for k,x in d.items() if isinstance(x,dict) and 'value' in x][:4])"; done
