bash tools/gpu.sh abn r03/single4 2 mpcium_amd/libmpcx.so,build/ab_s4/libmpcx.so --steps 1 --warmup 1 --extra-lines 0 --no-cpu-baseline --no-smi --keygen-sessions 4096 \
&& bash tools/gpu.sh envab r03/narrowkg 2 "MPCX_NARROW_ROUNDS=15" "MPCX_NARROW_ROUNDS=3" --steps 1 --warmup 1 --extra-lines 0 --no-cpu-baseline --no-smi --wallets 0 --keygen-sessions 4096
