# signing wallet pipelines (MPCX_SIGN_PIPELINE chunks,workers) with the shared host pool, interleaved
set -o pipefail
O=gpurun_out/pipe_ab
mkdir -p $O && export TMPDIR=/tmp
for pl in ${PIPES:-1,1 2,2 3,3 1,1 2,2 3,3}; do
  if [ "$pl" = default ]; then unset MPCX_SIGN_PIPELINE; else export MPCX_SIGN_PIPELINE=$pl; fi
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --extra-lines 0 --keygen-sessions 0 --no-cpu-baseline > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/ab.json'))
print('pipeline=$pl', *[f\"{k} {round(d[k]['value'],1)} busy {round(d[k]['engine_busy_s'],3)}\" for k in ('signing', 'signing_3_signers')])" | tee -a $O/ab.txt
done
