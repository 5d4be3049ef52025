# signing lines: the launch-time geometry model (default) vs the main geometry (+ matrix cores) at every size
set -o pipefail
O=gpurun_out/mx9; mkdir -p $O
for r in 1 2; do for v in model main; do
  if [ $v = model ]; then X=""; else X="--opt geom_policy=2"; fi
  timeout -k 10 500 python -u bench.py --steps 1 --warmup 1 --keygen-sessions 0 --extra-lines 0 --no-cpu-baseline $X --detail $O/d_${v}_$r.json > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail $O/b_${v}_$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/b_${v}_$r.json').read().strip().splitlines()[-1]); c=d['configs']
print('$v $r', d['value'], c['c4_sign']['value'], c['c4_sign_3_signers']['value'])"
done; done
