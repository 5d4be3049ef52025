bash tools/gpu.sh suite r03/s6 \
&& bash tools/gpu.sh envab r03/fbw 2 "MPCX_FB_WINDOW=8" "MPCX_FB_WINDOW=12" --steps 1 --warmup 1 --extra-lines 0 --no-cpu-baseline --no-smi --keygen-sessions 4096 \
&& bash tools/gpu.sh abn r03/wpe4 2 mpcium_amd/libmpcx.so,build/ab_wpe4/libmpcx.so --steps 1 --warmup 1 --extra-lines 0 --no-cpu-baseline --no-smi --keygen-sessions 4096 \
&& bash tools/gpu.sh pmc r03/pmc_valu "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES" --steps 2 --warmup 0 --wallets 0 --keygen-sessions 0 --no-cpu-baseline --no-smi \
&& bash tools/gpu.sh pmc r03/pmc_fetch "FETCH_SIZE" --steps 2 --warmup 0 --wallets 0 --keygen-sessions 0 --extra-lines 0 --no-cpu-baseline --no-smi \
&& bash tools/gpu.sh pmc r03/pmc_write "WRITE_SIZE" --steps 2 --warmup 0 --wallets 0 --keygen-sessions 0 --extra-lines 0 --no-cpu-baseline --no-smi \
&& bash tools/gpu.sh pmc r03/pmc_sign "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES" --steps 1 --warmup 0 --count 4096 --extra-lines 0 --keygen-sessions 0 --no-cpu-baseline --no-smi
