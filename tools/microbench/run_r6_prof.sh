# s_memtime phase profile of montmul_mx on the squaring-chain microbench (-DMX_PROF):
# cycles per squaring per phase, averaged over waves; 1 and 2 wavefronts per SIMD
set -o pipefail
O=gpurun_out/r06/prof; mkdir -p $O
cd tools/microbench
for v in prof profp; do for c in 16384 32768; do
  MX_PROF=1 MX_CHAIN_SO=mx_chain_r6$v.so timeout -k 10 60 python -u mx_chain.py $c 256 > ../../$O/${v}_${c}.json 2>/dev/null || exit 1
  echo "$v $c $(cat ../../$O/${v}_${c}.json | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['ok_mx'], d['ms_mx'], d.get('phase_cycles_per_squaring_mean_wave'), d.get('phase_cycles_total'))")"
done; done
