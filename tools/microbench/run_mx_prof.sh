# rocprofv3 kernel trace of the default bench (k_modexp_mx on) and the PMC passes of config 2
set -o pipefail
A="--steps 2 --warmup 0 --wallets 0 --keygen-sessions 0 --extra-lines 0 --no-cpu-baseline"
bash tools/gpu.sh pmc r05/pmc_mx_fetch "FETCH_SIZE" $A && \
bash tools/gpu.sh pmc r05/pmc_mx_write "WRITE_SIZE" $A && \
bash tools/gpu.sh pmc r05/pmc_mx_valu "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE SQ_INSTS_LDS" $A && \
python3 tools/pmc_kernels.py gpurun_out/r05/pmc_mx.json gpurun_out/r05/pmc_mx_fetch gpurun_out/r05/pmc_mx_write gpurun_out/r05/pmc_mx_valu --match k_modexp && \
bash tools/gpu.sh trace r05/trace_mx
