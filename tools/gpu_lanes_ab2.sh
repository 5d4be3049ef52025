# execution lanes 4 vs 8 (HW queues at HIP's default): signing / keygen lines, interleaved
set -o pipefail
O=gpurun_out/lanes_ab2
mkdir -p $O && export TMPDIR=/tmp
for ln in 4 8 4 8 4 8; do
  MPCX_LANES=$ln timeout -k 10 300 python bench.py --steps 1 --warmup 1 --extra-lines 0 --no-cpu-baseline > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/ab.json'))
print('lanes=$ln', *[f\"{k} {round(d[k]['value'],1)}\" for k in ('signing', 'signing_3_signers', 'keygen')])" | tee -a $O/ab.txt
done
