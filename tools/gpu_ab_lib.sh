# A/B two builds of libmpcx.so on one box: mpcium_amd/libmpcx.so (new) vs mpcium_amd/libmpcx_old.so,
# interleaved config-2 bench runs (4096-bit) and a 2048-bit line, after the GPU parity suite on the new build.
set -o pipefail
mkdir -p gpurun_out/ab && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/ab/pytest_gpu.txt; [ $rc -eq 0 ] || exit 1
cp mpcium_amd/libmpcx.so /tmp/libmpcx_new.so
for i in 1 2 3; do
  for v in new old; do
    cp /tmp/libmpcx_$v.so mpcium_amd/libmpcx.so 2>/dev/null || cp mpcium_amd/libmpcx_old.so mpcium_amd/libmpcx.so
    timeout -k 10 150 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --wallets 0 > gpurun_out/ab/b_${v}_$i.json 2>gpurun_out/ab/b_${v}_$i.err || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/ab/b_${v}_$i.json').read().strip().splitlines()[-1]);print('$v',$i,round(d['value']),round(d['roofline']['kernel_ms'],2))"
  done
done
cp /tmp/libmpcx_new.so mpcium_amd/libmpcx.so
