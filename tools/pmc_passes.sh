# Separate rocprofv3 --pmc passes over the bench workload (one counter group
# per pass; never combined with sys/runtime trace). Output: gpurun_out/pmc/<pass>/
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
run() { # name, counters...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o $name -- \
    python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --verify 0 --wallets 0 --keygen-sessions 0 --extra-lines 0 > $OUT/$name.log 2>&1
  local rc=$?; echo "pass $name rc=$rc"; return $rc
}
run fetch FETCH_SIZE && run write WRITE_SIZE && \
run valu SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU && \
run cycles SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU
