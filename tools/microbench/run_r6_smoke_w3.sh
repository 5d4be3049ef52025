# smoke (time it), then the 3-waves-per-SIMD A/B of config 2
set -o pipefail
O=gpurun_out/r06/$1; mkdir -p $O
export TMPDIR=/tmp
SECONDS=0; timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt; echo "smoke wall ${SECONDS} s"
bash tools/microbench/run_r6_libab.sh w3ab 2 base w3c6 w3c9
