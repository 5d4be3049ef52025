# concurrent ExpSet launches (+ AliceInit's Encrypt in the range proof's first
# launches): MtA / signing / proof GPU tests, then signing / keygen lines with
# MPCX_EXPSET_SERIAL=0 (concurrent) vs 1 (one launch after another), interleaved
set -o pipefail
O=gpurun_out/conc_ab
mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_mta.py tests/test_gpu_signing.py tests/test_gpu_proofs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pytest.txt | head -20; exit 1; }
for sr in 0 1 0 1; do
  MPCX_EXPSET_SERIAL=$sr timeout -k 10 300 python bench.py --steps 1 --warmup 1 --extra-lines 0 --no-cpu-baseline > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/ab.json'))
for key in ('signing', 'signing_3_signers', 'keygen'):
    s=d[key]; print('serial=$sr', key, round(s['value'],1), round(s['seconds'],3), 'busy', round(s['engine_busy_s'],3), s.get('rounds_s', ''))" | tee -a $O/ab.txt
done
