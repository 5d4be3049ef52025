bash tools/gpu.sh suite r03/final2 && bash tools/gpu.sh bench r03/final2b --steps 20 --warmup 5 \
&& bash tools/gpu.sh pmc r03/pmc_kg "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES" --steps 1 --warmup 0 --count 4096 --extra-lines 0 --wallets 0 --keygen-sessions 2048 --no-cpu-baseline --no-smi
