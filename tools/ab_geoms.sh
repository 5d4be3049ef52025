set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.txt; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_gpu.txt | head -20; exit 1; }
for cfg in "4096 2" "4096 6" "2048 1" "2048 5"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --modbits $1 --opt main_geom=$2 > gpurun_out/ab_$1_$2.json 2>gpurun_out/ab_$1_$2.err || { tail -5 gpurun_out/ab_$1_$2.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_$1_$2.json')); print('$1 geom $2', round(d['value']), 'frac', round(d['roofline']['frac'],3), d['config']['kernel_geometry'])"
done
