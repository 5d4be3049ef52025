# 2-rank rehearsal of the driver's scaling command on one GPU (both ranks share it)
set -o pipefail
mkdir -p gpurun_out/w2 && export TMPDIR=/tmp
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 2 --warmup 1 --wallets 2000 --keygen-sessions 32 --safe-primes 16 > gpurun_out/w2/bench.json 2> gpurun_out/w2/bench.err || { tail -30 gpurun_out/w2/bench.err; exit 1; }
test "$(grep -c . gpurun_out/w2/bench.json)" = 1 || { echo "stdout is not one line"; head -3 gpurun_out/w2/bench.json | cut -c1-120; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/w2/bench.json'))
print('n_gpus', d['n_gpus'], 'value', round(d['value']), 'digest', d.get('batch_digest',{}).get('match'), 'sub', [round(s['value']) for s in d.get('config2_per_operand_exponents',[])])
for k in ('signing','signing_3_signers','safe_prime','paillier_batch'):
    s=d.get(k); print(k, None if not s else (round(s['value'],1), s.get('n_gpus')))"
