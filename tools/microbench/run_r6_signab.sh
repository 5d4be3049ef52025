# Interleaved signing runs (2 and 3 signers, 10,000 wallets) of libmpcx variants:
#   bash tools/microbench/run_r6_signab.sh OUT ROUNDS variant...   (variants/<name>/libmpcx.so)
set -o pipefail
O=gpurun_out/r06/$1; R=$2; shift 2; mkdir -p $O
for r in $(seq 1 $R); do for v in "$@"; do
  MPCX_LIB_PATH=$(realpath variants/$v/libmpcx.so) timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --wallets 10000 \
      --keygen-sessions 0 --extra-lines 0 --no-cpu-baseline --no-smi --detail $O/${v}_$r.json > $O/${v}_$r.line 2> $O/${v}_$r.err \
      || { tail $O/${v}_$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${v}_$r.json')); print('$v', $r, round(d['signing']['value']), round(d['signing_3_signers']['value']), round(d['roofline']['kernel_ms'],2))"
done; done
