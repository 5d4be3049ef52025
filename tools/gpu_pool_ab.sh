# shared host thread pool (MPCX_HOST_POOL=1) vs a thread set per parallel loop (0):
# MtA / signing / proof / host GPU tests, then signing + keygen lines, interleaved
set -o pipefail
O=gpurun_out/pool_ab
mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_mta.py tests/test_gpu_signing.py tests/test_gpu_proofs.py tests/test_gpu_host.py -m gpu -x -q --timeout 250 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pytest.txt | head -20; exit 1; }
for v in 1 0 1 0 1 0 1 0; do
  MPCX_HOST_POOL=$v timeout -k 10 300 python bench.py --steps 1 --warmup 1 --extra-lines 0 --no-cpu-baseline > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/ab.json'))
print('pool=$v', *[f\"{k} {round(d[k]['value'],1)}\" for k in ('signing', 'signing_3_signers', 'keygen')], 'cpu', round(d['signing']['host_cpu_s'],1), round(d['signing_3_signers']['host_cpu_s'],1))" | tee -a $O/ab.txt
done
