# signing: chain start stagger sweep, interleaved
set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
for st in 0 40 100 0 40 100 200; do
  MPCX_SIGN_STAGGER_MS=$st timeout -k 10 300 python bench.py --steps 1 --warmup 1 --extra-lines 0 --keygen-sessions 0 --no-cpu-baseline > gpurun_out/stg.json 2> gpurun_out/stg.err || { tail gpurun_out/stg.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/stg.json'))
print('stagger=$st', 'sign2', round(d['signing']['value']), round(d['signing']['engine_busy_s'],3), 'sign3', round(d['signing_3_signers']['value']))"
done
