# GPU suite + smoke on the current tree (round 6)
set -o pipefail
O=gpurun_out/r06/$1; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -3 $O/pytest_gpu.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pytest_gpu.txt | head -20; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
