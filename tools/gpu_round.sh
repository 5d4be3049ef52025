set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.txt
if [ $rc -ne 0 ]; then exit 1; fi
timeout -k 10 400 python tools/ab_variants.py run 3 > gpurun_out/ab.txt 2>&1
rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab.txt
if [ $rc -ne 0 ]; then exit 1; fi
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-seconds 10 > gpurun_out/bench.txt 2>&1
echo "bench rc=$?"; tail -1 gpurun_out/bench.txt
