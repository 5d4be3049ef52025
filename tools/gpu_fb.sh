set -o pipefail
mkdir -p gpurun_out/fb && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_modexp.py -x -v --timeout 120 --timeout-method thread -k "fixed_base or window_sched" > gpurun_out/fb/pytest.txt 2>&1
rc=$?; tail -4 gpurun_out/fb/pytest.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python tools/fixedbase_bench.py > gpurun_out/fb/bench.json 2>gpurun_out/fb/bench.err || { tail gpurun_out/fb/bench.err; exit 1; }
cat gpurun_out/fb/bench.json
