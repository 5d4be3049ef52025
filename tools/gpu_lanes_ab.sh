# execution lanes x HW queues: signing / keygen lines, interleaved
set -o pipefail
O=gpurun_out/lanes_ab
mkdir -p $O && export TMPDIR=/tmp
for cfg in "4 4" "8 8" "8 4" "4 4" "8 8" "8 4"; do
  set -- $cfg
  MPCX_LANES=$1 GPU_MAX_HW_QUEUES=$2 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --extra-lines 0 --no-cpu-baseline > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/ab.json'))
print('lanes=$1 hwq=$2 config2', round(d['value']))
for key in ('signing', 'signing_3_signers', 'keygen'):
    s=d[key]; print('lanes=$1 hwq=$2', key, round(s['value'],1), round(s['seconds'],3), 'busy', round(s['engine_busy_s'],3))" | tee -a $O/ab.txt
done
