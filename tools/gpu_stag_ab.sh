# 2 half-wallet pipelines (the 2-signer default): start stagger of the second pipeline, interleaved
set -o pipefail
O=gpurun_out/stag_ab
mkdir -p $O && export TMPDIR=/tmp
for st in 0 60 150 0 60 150 0 60 150; do
  MPCX_SIGN_CHUNK_STAGGER_MS=$st timeout -k 10 300 python bench.py --steps 1 --warmup 1 --extra-lines 0 --keygen-sessions 0 --no-cpu-baseline > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/ab.json'))
print('stagger=$st', *[f\"{k} {round(d[k]['value'],1)} busy {round(d[k]['engine_busy_s'],3)}\" for k in ('signing', 'signing_3_signers')])" | tee -a $O/ab.txt
done
