# Squaring-chain microbench (mx_chain.py): full montmul_mx, product loop alone
# (MPCX_MX_TIMING=1), reduction alone (=2), at 1, 2 and 4 wavefronts per SIMD
set -o pipefail
O=gpurun_out/r06/occ; mkdir -p $O
cd tools/microbench
for v in full prod red; do for c in 16384 32768 65536; do
  MX_CHAIN_SO=mx_chain_r6$v.so timeout -k 10 120 python -u mx_chain.py $c 256 > ../../$O/${v}_$c.json 2>/dev/null || exit 1
  echo "$v $c $(python3 -c "import json; d=json.load(open('../../$O/${v}_$c.json')); print(d['ok_mx'], d['ms_mx'], d['ms_cios'])")"
done; done
