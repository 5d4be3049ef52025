mkdir -p gpurun_out/prof_r01 && export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu3.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu3.txt
if [ $rc -ne 0 ]; then exit 1; fi
timeout -k 10 400 python tools/ab_variants.py run 3 > gpurun_out/ab.txt 2>&1
rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab.txt
if [ $rc -ne 0 ]; then exit 1; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r01 -o r01 -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r01/bench.txt 2>&1
echo "prof rc=$?"; tail -2 gpurun_out/prof_r01/bench.txt; find gpurun_out/prof_r01 -name "*stats*" -exec cat {} \; 
