# blocking-sync waits and pinned staging vs spin / pageable: signing and keygen lines, interleaved
set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
for cfg in "0 1" "1 0" "0 1" "1 0" "1 1" "0 0"; do
  set -- $cfg
  MPCX_SPIN_WAIT=$1 MPCX_PINNED=$2 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --extra-lines 0 --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/ab.json'))
print('spin=$1 pinned=$2', 'sign2', round(d['signing']['value']), 'sign3', round(d['signing_3_signers']['value']), 'keygen', round(d['keygen']['value'],1), 'cpu2', round(d['signing']['host_cpu_s'],1))"
done
