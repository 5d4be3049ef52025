# carry-pass skip (MX_CARRY_SKIP=1): squaring chains checked against pow, then config 2 A/B (digest checked)
set -o pipefail
O=gpurun_out/r06/cskip; mkdir -p $O
cd tools/microbench
for v in base cskip; do
  MX_CHAIN_SO=mx_chain_r6$v.so timeout -k 10 60 python -u mx_chain.py 65536 256 > ../../$O/chain_${v}.json 2>/dev/null || exit 1
  echo "chain $v $(python3 -c "import json; d=json.load(open('../../$O/chain_${v}.json')); print(d['ok_mx'], d['mx_values_ge_2m'], d['mx_max_digit'], d['ms_mx'])")"
done
cd ../..
bash tools/microbench/run_r6_libab.sh cskipab 3 def cskip
