set -o pipefail
O=gpurun_out/r06/e1; mkdir -p $O
bash tools/gpu.sh ab r06/e1 3 variants/e0/libmpcx.so mpcium_amd/libmpcx.so --steps 5 --warmup 1 --wallets 0 --keygen-sessions 0 --extra-lines 0 --no-cpu-baseline --verify 16
