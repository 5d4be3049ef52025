bash tools/gpu.sh envab r03/pipes 3 "MPCX_SIGN_PIPELINE=3,3" "MPCX_SIGN_PIPELINE=2,2" --steps 1 --warmup 1 --extra-lines 0 --no-cpu-baseline --no-smi --keygen-sessions 0 \
&& bash tools/gpu.sh envab r03/lanes 3 "MPCX_LANES=6" "MPCX_LANES=4" --steps 1 --warmup 1 --extra-lines 0 --no-cpu-baseline --no-smi --keygen-sessions 0
