bash tools/gpu.sh envab r03/pipes3 4 "MPCX_SIGN_PIPELINE=1,1" "MPCX_SIGN_PIPELINE=2,2" --steps 1 --warmup 1 --extra-lines 0 --no-cpu-baseline --no-smi --keygen-sessions 0 --signers 3
