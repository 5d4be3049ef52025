# What independent work costs inside the product loop (mx_chain.hip, product loop
# alone): 1 dummy i8 MFMA per row step (148 per product); 3 per row step with a
# scheduling fence per row step (444 per product, ~ the reduction's 417), against
# the product loop alone with and without the fence; full montmul_mx with the fence
set -o pipefail
O=gpurun_out/r06/dummy2; mkdir -p $O
cd tools/microbench
for r in 1 2; do for v in prod prodf dm1 dm3f full fullf; do for c in 16384 32768; do
  MX_CHAIN_SO=mx_chain_r6$v.so timeout -k 10 60 python -u mx_chain.py $c 256 > ../../$O/${v}_${c}_$r.json 2>/dev/null || exit 1
  echo "$v $c $r $(python3 -c "import json; d=json.load(open('../../$O/${v}_${c}_$r.json')); print(d['ok_mx'], d['ms_mx'])")"
done; done; done
