set -o pipefail
mkdir -p gpurun_out/sg && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_mta.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sg/pytest.txt 2>&1
rc=$?; tail -2 gpurun_out/sg/pytest.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 1 --no-cpu-baseline --count 4096 > gpurun_out/sg/bench.json 2>gpurun_out/sg/b.err || { tail gpurun_out/sg/b.err; exit 1; }
python -c "
import json
d=json.loads(open('gpurun_out/sg/bench.json').read().strip().splitlines()[-1])['signing']; print(round(d['value']), d['seconds'], d['engine_busy_s'], d['rounds_s'])"
