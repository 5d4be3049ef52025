# One GPU call: parity suite with 6-bit sliding windows (33-entry tables),
# then the config-2 kernel with the window cap at 5 vs 6 (4096- and 2048-bit).
set -o pipefail
mkdir -p gpurun_out/w6 && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/w6/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/w6/pytest_gpu.txt; [ $rc -eq 0 ] || exit 1
for w in 5 6 5 6; do
  for mb in 4096 2048; do
    timeout -k 10 120 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --wallets 0 --keygen-sessions 0 --extra-lines 0 --modbits $mb --opt sched_width=$w > gpurun_out/w6/b${mb}_w$w.json 2> gpurun_out/w6/b.err || { tail gpurun_out/w6/b.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/w6/b${mb}_w$w.json').read().strip().splitlines()[-1]); print('w=$w mod=$mb', round(d['value']), round(d['roofline']['kernel_ms'],2), round(d['roofline']['frac'],4))"
  done
done
