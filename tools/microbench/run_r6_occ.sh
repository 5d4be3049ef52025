# Squaring-chain microbench (mx_chain.py): full montmul_mx, product loop alone
# (MPCX_MX_TIMING=1), reduction alone (=2), at 1, 2 and 4 wavefronts per SIMD;
# then two PMC passes of each variant at 65,536 operands
set -o pipefail
O=gpurun_out/r06/occ; mkdir -p $O
export TMPDIR=/tmp
cd tools/microbench
for v in full prod red; do for c in 16384 32768 65536; do
  MX_CHAIN_SO=mx_chain_r6$v.so timeout -k 10 120 python -u mx_chain.py $c 256 > ../../$O/${v}_$c.json 2>/dev/null || exit 1
  echo "$v $c $(python3 -c "import json; d=json.load(open('../../$O/${v}_$c.json')); print(d['ok_mx'], d['ms_mx'], d['ms_cios'])")"
done; done
for v in full prod red; do
  MX_CHAIN_SO=mx_chain_r6$v.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY --output-format csv -d ../../$O/pmc_${v}_a -o pmc -- python3 mx_chain.py 65536 64 > /dev/null 2> ../../$O/pmc_${v}_a.err || exit 1
  MX_CHAIN_SO=mx_chain_r6$v.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d ../../$O/pmc_${v}_b -o pmc -- python3 mx_chain.py 65536 64 > /dev/null 2> ../../$O/pmc_${v}_b.err || exit 1
done
cd ../..
python3 tools/pmc_chain.py $O
