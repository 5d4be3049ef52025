mkdir -p gpurun_out/r03/c \
&& timeout -k 10 600 python -u -m pytest tests/test_gpu_modexp.py tests/test_gpu_mta.py tests/test_gpu_proofs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03/c/pytest.txt 2>&1 \
&& tail -2 gpurun_out/r03/c/pytest.txt \
&& bash tools/gpu.sh abn r03/pf 2 mpcium_amd/libmpcx.so,build/ab_nopf/libmpcx.so --steps 1 --warmup 1 --extra-lines 0 --no-cpu-baseline --no-smi --keygen-sessions 4096
