# the GPU modules from test_gpu_proofs on (alphabetical order of the suite), smoke, then
# the 3-waves-per-SIMD A/B of config 2
set -o pipefail
O=gpurun_out/r06/$1; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_proofs.py tests/test_gpu_signing.py tests/test_gpu_wire.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu_rest.txt 2>&1
rc=$?; tail -3 $O/pytest_gpu_rest.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pytest_gpu_rest.txt | head -20; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
bash tools/microbench/run_r6_libab.sh w3ab 2 base w3c6 w3c9
