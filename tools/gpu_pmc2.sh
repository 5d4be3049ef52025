# config-3 batch-size sweep, then PMC passes (one counter group per run) over
# the config-2 + config-3 bench lines
set -o pipefail
mkdir -p gpurun_out/pmc2 && export TMPDIR=/tmp
for b in 262144 393216 524288 786432; do
  MPCX_SAFEPRIME_BATCH=$b timeout -k 10 300 python bench.py --steps 1 --warmup 0 --count 4096 --wallets 0 --keygen-sessions 0 --no-cpu-baseline > gpurun_out/sp_b$b.json 2> gpurun_out/sp_b$b.err || { tail gpurun_out/sp_b$b.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/sp_b$b.json'))['safe_prime']; print('batch $b', round(d['value'],1), 'primes/s', round(d['fermat_tests_per_s']/1e6,3), 'M tests/s', round(d['seconds'],4), d['fermat_tests'])"
done
i=0
for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $pass --output-format csv -d gpurun_out/pmc2/p$i -o pmc -- python3 bench.py --steps 2 --warmup 0 --wallets 0 --keygen-sessions 0 --no-cpu-baseline > gpurun_out/pmc2/p$i.json 2> gpurun_out/pmc2/p$i.err || { tail gpurun_out/pmc2/p$i.err; exit 1; }
  echo "pass $i done"
done
ls -R gpurun_out/pmc2 | head -30
