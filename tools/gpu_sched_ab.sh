set -o pipefail
mkdir -p gpurun_out/s1 && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s1/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/s1/pytest_gpu.txt; [ $rc -eq 0 ] || exit 1
for w in 0 5 4; do
  timeout -k 10 200 python bench.py --steps 3 --no-cpu-baseline --wallets 0 --opt sched_width=$w > gpurun_out/s1/b4096_w$w.json 2>gpurun_out/s1/b.err || exit 1
  timeout -k 10 200 python bench.py --steps 3 --no-cpu-baseline --wallets 0 --modbits 2048 --opt sched_width=$w > gpurun_out/s1/b2048_w$w.json 2>gpurun_out/s1/b.err || exit 1
done
python - <<'P'
import json,glob
for f in sorted(glob.glob("gpurun_out/s1/b*_w*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, round(d["value"]), d["roofline"]["kernel_ms"])
P
