set -o pipefail
mkdir -p gpurun_out/fb2 && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_mta.py tests/test_gpu_proofs.py tests/test_gpu_host.py -x -v --timeout 120 --timeout-method thread > gpurun_out/fb2/pytest.txt 2>&1
rc=$?; tail -4 gpurun_out/fb2/pytest.txt; [ $rc -eq 0 ] || exit 1
MPCX_FIXED_BASE=0 timeout -k 10 200 python bench.py --steps 1 --no-cpu-baseline --count 4096 > gpurun_out/fb2/bench_fb0.json 2>gpurun_out/fb2/b.err || { tail gpurun_out/fb2/b.err; exit 1; }
timeout -k 10 200 python bench.py --steps 1 --no-cpu-baseline --count 4096 > gpurun_out/fb2/bench_fb1.json 2>gpurun_out/fb2/b.err || { tail gpurun_out/fb2/b.err; exit 1; }
python -c "
import json
for f in ('fb0','fb1'):
    d=json.loads(open('gpurun_out/fb2/bench_%s.json'%f).read().strip().splitlines()[-1])['signing']; print(f, round(d['value']), d['rounds_s'])"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fb2/prof -o fb -- python3 tools/fixedbase_bench.py 16384 > gpurun_out/fb2/prof_fb.json 2>gpurun_out/fb2/prof.err || { tail gpurun_out/fb2/prof.err; exit 1; }
find gpurun_out/fb2/prof -name '*kernel_stats*' -exec cat {} \;
