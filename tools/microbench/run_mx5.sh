# workgroup size / wave stagger sweep of the chain microbench
set -o pipefail
O=gpurun_out/mx5; mkdir -p $O
cd tools/microbench
for v in mx_chain.so mx_chain_w8.so mx_chain_w8s1.so mx_chain_w8s2.so mx_chain_w8s3.so mx_chain_w4s2.so mx_chain.so; do
  MX_CHAIN_SO=$v timeout -k 10 120 python -u mx_chain.py 65536 256 > ../../$O/$v.json 2>/dev/null || exit 1
  echo "$v $(python3 -c "import json; d=json.load(open('../../$O/$v.json')); print(d['ok_mx'], d['ns_per_squaring_mx'], d['ns_per_squaring_cios'], d['speedup'])")"
done
