# the driver's default bench on the final tree + its config-2 trace, then 3 more mx_seg_min rounds
set -o pipefail
bash tools/microbench/run_r6_final.sh final2 && \
bash tools/gpu.sh argab r06/segmin2 3 "--opt mx_seg_min=256" "--opt mx_seg_min=64" --steps 1 --warmup 1 --extra-lines 0 --no-cpu-baseline --keygen-sessions 8192
