# Interleaved keygen (8,192 sessions) + 2-signer signing runs of libmpcx variants:
#   bash tools/microbench/run_r6_fbab.sh OUT ROUNDS variant...   (variants/<name>/libmpcx.so)
set -o pipefail
O=gpurun_out/r06/$1; R=$2; shift 2; mkdir -p $O
for r in $(seq 1 $R); do for v in "$@"; do
  MPCX_LIB_PATH=$(realpath variants/$v/libmpcx.so) timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --wallets 10000 --no-sign3 \
      --keygen-sessions 8192 --extra-lines 0 --no-cpu-baseline --no-smi --detail $O/${v}_$r.json > $O/${v}_$r.line 2> $O/${v}_$r.err \
      || { tail $O/${v}_$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${v}_$r.json')); print('$v', $r, round(d['keygen']['value'],1), round(d['signing']['value']))"
done; done
