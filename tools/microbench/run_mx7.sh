# MX tuning sweep on the squaring-chain microbench (interleaved, base twice)
set -o pipefail
O=gpurun_out/mx7; mkdir -p $O
cd tools/microbench
for v in mx_chain.so mx_chain_nf.so mx_chain_cs19.so mx_chain_prio.so mx_chain_cs10.so mx_chain.so mx_chain_cs19.so mx_chain_prio.so; do
  MX_CHAIN_SO=$v timeout -k 10 120 python -u mx_chain.py 65536 256 > ../../$O/$v.json 2>/dev/null || exit 1
  echo "$v $(python3 -c "import json; d=json.load(open('../../$O/$v.json')); print(d['ok_mx'], d['ns_per_squaring_mx'], d['ns_per_squaring_cios'], d['speedup'])")"
done
