# Phase pairing on the squaring-chain microbench: 8-wave workgroups, the second
# half one phase (product loop / reduction) behind the first (MX_PHASE_BARRIER)
set -o pipefail
O=gpurun_out/r06/pb; mkdir -p $O
cd tools/microbench
for r in 1 2; do for v in b4 b8 pb8 pb8p; do for c in 32768 65536; do
  MX_CHAIN_SO=mx_chain_r6$v.so timeout -k 10 60 python -u mx_chain.py $c 256 > ../../$O/${v}_${c}_$r.json 2>/dev/null || exit 1
  echo "$v $c $r $(python3 -c "import json; d=json.load(open('../../$O/${v}_${c}_$r.json')); print(d['ok_mx'], d['ms_mx'], d['ms_cios'])")"
done; done; done
