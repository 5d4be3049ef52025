# Pipelined reduction (MX_PIPE: a chunk's normalisation under the next chunk's
# MFMAs) vs MX_PIPE=0, chunk sizes 13 / 10 / 7; phase profiles (-DMX_PROF)
set -o pipefail
O=gpurun_out/r06/pipe; mkdir -p $O
cd tools/microbench
for r in 1 2; do for v in np p13 p10 p7; do for c in 16384 65536; do
  MX_CHAIN_SO=mx_chain_r6$v.so timeout -k 10 60 python -u mx_chain.py $c 256 > ../../$O/${v}_${c}_$r.json 2>/dev/null || exit 1
  echo "$v $c $r $(python3 -c "import json; d=json.load(open('../../$O/${v}_${c}_$r.json')); print(d['ok_mx'], d['ms_mx'])")"
done; done; done
for v in p13prof p7prof; do for c in 16384 32768; do
  MX_PROF=1 MX_CHAIN_SO=mx_chain_r6$v.so timeout -k 10 60 python -u mx_chain.py $c 256 > ../../$O/${v}_${c}.json 2>/dev/null || exit 1
  echo "$v $c $(cat ../../$O/${v}_${c}.json | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['ok_mx'], d['ms_mx'], d.get('phase_cycles_per_squaring_mean_wave'), d.get('phase_cycles_total'))")"
done; done
