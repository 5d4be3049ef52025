# MX_SPLIT_MAD=1 (default now): the matrix-core GPU tests, then config 2 against the round-6 base library
set -o pipefail
O=gpurun_out/r06/smadlib; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_mx.py tests/test_gpu_modexp.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
bash tools/microbench/run_r6_libab.sh smadab 3 base smad
