# geometry-5 MX: GPU parity tests, then the 2048-bit config-2 shape and a keygen mix with and without MX
set -o pipefail
O=gpurun_out/mx6; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_mx.py -x -q --timeout 380 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for mx in 1 0; do
  timeout -k 10 300 python -u bench.py --modbits 2048 --steps 5 --warmup 2 --extra-lines 0 --wallets 0 --keygen-sessions 0 --no-cpu-baseline --opt mx=$mx --detail $O/d2048_mx$mx.json > $O/b2048_mx$mx.json 2> $O/b2048_mx$mx.err || { tail $O/b2048_mx$mx.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b2048_mx$mx.json').read().strip().splitlines()[-1]); print('2048 mx=$mx', d['value'], d['ms_per_step'])"
done
for mx in 1 0 1 0; do
  timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --extra-lines 0 --wallets 0 --keygen-sessions 12288 --no-cpu-baseline --opt mx=$mx --detail $O/dkg_mx$mx.json > $O/bkg_mx$mx.json 2> $O/bkg_mx$mx.err || { tail $O/bkg_mx$mx.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bkg_mx$mx.json').read().strip().splitlines()[-1]); print('keygen mx=$mx', d['configs']['c5_keygen']['value'], 'c2', d['value'])"
done
