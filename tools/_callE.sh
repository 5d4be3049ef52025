mkdir -p gpurun_out/r03/world2 \
&& timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/r03/world2/bench.json 2> gpurun_out/r03/world2/bench.err \
&& python3 -c "import json; d=json.load(open('gpurun_out/r03/world2/bench.json')); print('world2', d['n_gpus'], round(d['value']), d.get('batch_digest',{}).get('match'), round(d['signing']['value']), round(d['safe_prime']['value'],1))" \
&& bash tools/gpu.sh envab r03/narrow 3 "MPCX_NARROW_ROUNDS=15" "MPCX_NARROW_ROUNDS=3" --steps 1 --warmup 1 --extra-lines 0 --no-cpu-baseline --no-smi --keygen-sessions 0 \
&& bash tools/gpu.sh envab r03/coal 2 "MPCX_COALESCE=3" "MPCX_COALESCE=2" --steps 1 --warmup 1 --extra-lines 0 --no-cpu-baseline --no-smi --keygen-sessions 0 \
&& bash tools/gpu.sh abn r03/fence 2 mpcium_amd/libmpcx.so,build/ab_f2/libmpcx.so,build/ab_f0/libmpcx.so --steps 1 --warmup 1 --wallets 0 --keygen-sessions 0 --no-cpu-baseline --no-smi
