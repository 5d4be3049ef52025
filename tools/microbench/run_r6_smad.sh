# the reduction's digit split on the MAD pipe (MX_SPLIT_MAD=1) vs the VALU split, squaring-chain microbench
set -o pipefail
O=gpurun_out/r06/smad; mkdir -p $O
cd tools/microbench
for r in 1 2; do for v in base smad; do for c in 16384 65536; do
  MX_CHAIN_SO=mx_chain_r6$v.so timeout -k 10 60 python -u mx_chain.py $c 256 > ../../$O/${v}_${c}_$r.json 2>/dev/null || exit 1
  echo "$v $c $r $(python3 -c "import json; d=json.load(open('../../$O/${v}_${c}_$r.json')); print(d['ok_mx'], d['mx_values_ge_2m'], d['ms_mx'])")"
done; done; done
