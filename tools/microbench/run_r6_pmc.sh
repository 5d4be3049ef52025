# PMC passes of config 2 on the round-6 tree (one counter group per run), reduced per kernel
set -o pipefail
A="--steps 2 --warmup 0 --wallets 0 --keygen-sessions 0 --extra-lines 0 --no-cpu-baseline --no-smi"
bash tools/gpu.sh pmc r06/pmc_fetch "FETCH_SIZE" $A && \
bash tools/gpu.sh pmc r06/pmc_write "WRITE_SIZE" $A && \
bash tools/gpu.sh pmc r06/pmc_valu "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_VALU" $A && \
bash tools/gpu.sh pmc r06/pmc_wait "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" $A && \
python3 tools/pmc_kernels.py gpurun_out/r06/pmc_mx.json gpurun_out/r06/pmc_fetch gpurun_out/r06/pmc_write gpurun_out/r06/pmc_valu gpurun_out/r06/pmc_wait --match k_modexp && cat gpurun_out/r06/pmc_mx.json | head -60
