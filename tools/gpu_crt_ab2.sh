# AliceEnd verification by CRT (MPCX_VERIFY_CRT=1) vs mod N^2 (0): signing lines, 5 interleaved pairs
set -o pipefail
O=gpurun_out/crt_ab2
mkdir -p $O && export TMPDIR=/tmp
for v in 1 0 1 0 1 0 1 0 1 0; do
  MPCX_VERIFY_CRT=$v timeout -k 10 300 python bench.py --steps 1 --warmup 1 --extra-lines 0 --keygen-sessions 0 --no-cpu-baseline > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/ab.json'))
print('crt=$v', *[f\"{k} {round(d[k]['value'],1)} busy {round(d[k]['engine_busy_s'],3)}\" for k in ('signing', 'signing_3_signers')])" | tee -a $O/ab.txt
done
