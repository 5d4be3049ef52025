# kernel trace of the config-3 line (short config-2 batch, no signing / keygen)
set -o pipefail
O=gpurun_out/sp_trace
mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o sp -- python3 bench.py --steps 1 --warmup 0 --count 4096 --wallets 0 --keygen-sessions 0 --no-cpu-baseline > $O/sp.json 2> $O/sp.err || { tail $O/sp.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/sp.json'))['safe_prime']; print(round(d['value'],1), round(d['seconds'],4))"
