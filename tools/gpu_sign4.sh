# signing: one pipeline vs two half-batch pipelines (interleaved)
set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
for pl in 1,1 2,2 1,1 2,2; do
  MPCX_SIGN_PIPELINE=$pl timeout -k 10 300 python bench.py --steps 1 --warmup 1 --extra-lines 0 --keygen-sessions 0 --no-cpu-baseline > gpurun_out/sign_pl.json 2> gpurun_out/sign_pl.err || { tail gpurun_out/sign_pl.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/sign_pl.json'))
for key in ('signing', 'signing_3_signers'):
    s=d[key]; print('$pl', key, round(s['value']), round(s['seconds'],3), 'busy', round(s['engine_busy_s'],3), 'cpu', round(s['host_cpu_s'],1))"
done
