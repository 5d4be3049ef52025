# One GPU call: new F4 wire + sharded safe-prime parity tests, then a 2-rank
# rehearsal of the multi-GPU bench path on one GPU (both ranks on cuda:0).
set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_host.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_f4.txt 2>&1
rc=$?; tail -15 gpurun_out/pytest_f4.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --count 16384 --wallets 1000 --keygen-sessions 0 --no-cpu-baseline > gpurun_out/bench_w2.json 2> gpurun_out/bench_w2.err || { tail -30 gpurun_out/bench_w2.err; exit 1; }
cat gpurun_out/bench_w2.json
