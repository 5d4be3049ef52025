# N = 2 rehearsals on one GPU: the driver's torchrun path (two ranks sharing the
# GPU) and mpcium's one-process node shape with two logical devices
set -o pipefail
O=gpurun_out/r06/n2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py --gpus 2 --steps 3 --warmup 1 --wallets 2000 --keygen-sessions 2048 --detail $O/bench_detail.json > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['n_gpus'], d['value'], d.get('digest_match'), {k: v['value'] for k, v in d.get('configs', {}).items()})"
timeout -k 10 500 python3 bench.py --node --node-dup 2 --steps 3 --warmup 1 --wallets 2000 --keygen-sessions 2048 --detail $O/node_detail.json > $O/node.json 2> $O/node.err || { tail $O/node.err; exit 1; }
head -c 1500 $O/node.json
