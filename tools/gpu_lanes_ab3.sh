# execution lanes 4 vs 6 for the signing lines (keygen keeps its 8-lane budget), interleaved
set -o pipefail
O=gpurun_out/lanes_ab3
mkdir -p $O && export TMPDIR=/tmp
for ln in 4 6 4 6 4 6 4 6; do
  MPCX_LANES=$ln timeout -k 10 300 python bench.py --steps 1 --warmup 1 --extra-lines 0 --keygen-sessions 0 --no-cpu-baseline > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/ab.json'))
print('lanes=$ln', *[f\"{k} {round(d[k]['value'],1)} busy {round(d[k]['engine_busy_s'],3)}\" for k in ('signing', 'signing_3_signers')])" | tee -a $O/ab.txt
done
