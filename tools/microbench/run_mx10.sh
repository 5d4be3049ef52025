# product-loop emission (raw low word, masked after the lane shift: MX_EMIT_RAW) and the
# 64-bit digit sum (MX_SPLIT64) on the squaring-chain microbench (interleaved, twice);
# both neutral or slower, the knobs were not kept
set -o pipefail
O=gpurun_out/r05/mx10; mkdir -p $O
cd tools/microbench
for r in 1 2; do for v in base raw s64 both; do
  MX_CHAIN_SO=mx_chain_$v.so timeout -k 10 120 python -u mx_chain.py 65536 256 > ../../$O/${v}_$r.json 2>/dev/null || exit 1
  echo "$v $r $(python3 -c "import json; d=json.load(open('../../$O/${v}_$r.json')); print(d['ok_mx'], d['ns_per_squaring_mx'], d['ns_per_squaring_cios'], d['speedup'])")"
done; done
