# Two separate --pmc passes (FETCH_SIZE, WRITE_SIZE) over the bench's main
# kernel only, then the per-launch summary. Output under gpurun_out/pmc/.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
run() {
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o $name -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --verify 0 --wallets 0 --keygen-sessions 0 --extra-lines 0 > $OUT/$name.log 2>&1
  local rc=$?; echo "pass $name rc=$rc"; return $rc
}
run fetch FETCH_SIZE && run write WRITE_SIZE && python3 tools/pmc_summary.py gpurun_out/pmc > $OUT/summary.json && cat $OUT/summary.json
