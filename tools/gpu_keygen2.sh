# config-5 line: proof chains vs prove-then-verify barrier, interleaved
set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
for c in 1 0 1 0 1 0; do
  MPCX_KEYGEN_CHAINS=$c timeout -k 10 300 python bench.py --steps 1 --warmup 1 --wallets 0 --extra-lines 0 --no-cpu-baseline > gpurun_out/kg.json 2> gpurun_out/kg.err || { tail gpurun_out/kg.err; exit 1; }
  python -c "
import json; s=json.load(open('gpurun_out/kg.json'))['keygen']; print('chains=$c', round(s['value'],1), round(s['seconds'],3), round(s.get('engine_busy_s'),3))"
done
