# keygen/reshare mix: the launch-time geometry model (default) vs the main geometry at every size
set -o pipefail
O=gpurun_out/kgpol; mkdir -p $O
for r in 1 2; do for v in model main; do
  if [ $v = model ]; then X=""; else X="--opt geom_policy=2"; fi
  timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --extra-lines 0 --wallets 0 --keygen-sessions 12288 --no-cpu-baseline $X --detail $O/d_${v}_$r.json > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail $O/b_${v}_$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/b_${v}_$r.json').read().strip().splitlines()[-1]); c=d['configs']
print('$v $r', c['c5_keygen']['value'])"
done; done
