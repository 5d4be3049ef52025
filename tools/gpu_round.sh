set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.txt
if [ $rc -ne 0 ]; then exit 1; fi
for opt in "split=1" "split=0"; do
for c in 27648 65536 82944 8192 1024; do
  timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --count $c --opt $opt > gpurun_out/bench_$opt_c$c.txt 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_$opt_c$c.txt').read().strip().splitlines()[-1]); print('$opt', $c, round(d['value']), round(d['roofline']['kernel_ms'],2))"
done
done
