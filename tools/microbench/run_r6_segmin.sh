# node-mode line check, then mx_seg_min 256 (default) vs 64 on signing + keygen, 3 interleaved rounds
set -o pipefail
O=gpurun_out/r06/segmin; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_multidev.py -m gpu -x -q -k node_mode --timeout 500 --timeout-method thread > $O/node_test.txt 2>&1 || { tail -30 $O/node_test.txt; exit 1; }
tail -2 $O/node_test.txt
bash tools/gpu.sh argab r06/segmin 3 "--opt mx_seg_min=256" "--opt mx_seg_min=64" --steps 1 --warmup 1 --extra-lines 0 --no-cpu-baseline --keygen-sessions 8192
