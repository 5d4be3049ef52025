mkdir -p gpurun_out/r03/g7 \
&& timeout -k 10 600 python -u -m pytest tests/test_gpu_modexp.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03/g7/pytest_modexp.txt 2>&1 && tail -1 gpurun_out/r03/g7/pytest_modexp.txt \
&& MPCX_MAIN_GEOM0=7 timeout -k 10 600 python -u -m pytest tests/test_gpu_proofs.py tests/test_gpu_signing.py tests/test_gpu_primes.py -m gpu -x -q --timeout 300 --timeout-method thread -k "keygen or mod or fac or dln or preparams or safe" > gpurun_out/r03/g7/pytest_geom7.txt 2>&1 && tail -1 gpurun_out/r03/g7/pytest_geom7.txt \
&& bash tools/gpu.sh envab r03/g7ab 2 "MPCX_MAIN_GEOM0=0" "MPCX_MAIN_GEOM0=7" --steps 1 --warmup 1 --extra-lines 0 --no-cpu-baseline --no-smi --wallets 0 --keygen-sessions 4096
