# keygen line: the driver's 8-lane budget vs 4 lanes (MPCX_KEYGEN_LANES), interleaved; signing unchanged alongside
set -o pipefail
O=gpurun_out/kg_ab
mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_proofs.py tests/test_gpu_signing.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pytest.txt | head -20; exit 1; }
for kl in 8 4 8 4 8 4; do
  MPCX_KEYGEN_LANES=$kl timeout -k 10 300 python bench.py --steps 1 --warmup 1 --extra-lines 0 --no-cpu-baseline > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/ab.json'))
print('keygen_lanes=$kl', *[f\"{k} {round(d[k]['value'],1)}\" for k in ('signing', 'signing_3_signers', 'keygen')])" | tee -a $O/ab.txt
done
