# coalescer fill wait (MPCX_COALESCE_MIN_OPS) on keygen/reshare and 2-signer signing: 0 (default) vs 4096 vs 16384,
# three interleaved rounds; one bench process per arm and round
set -o pipefail
O=gpurun_out/cmin; mkdir -p $O
for r in 1 2 3; do for v in 0 4096 16384; do
  MPCX_COALESCE_MIN_OPS=$v timeout -k 10 420 python -u bench.py --steps 1 --warmup 1 --extra-lines 0 --wallets 10000 --no-sign3 \
    --keygen-sessions 12288 --no-cpu-baseline --no-smi --detail $O/d_${v}_$r.json > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err \
    || { tail $O/b_${v}_$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/b_${v}_$r.json').read().strip().splitlines()[-1]); c=d['configs']
print('min_ops=$v round $r', 'keygen', c['c5_keygen']['value'], 'sign2', c['c4_sign']['value'])"
done; done
