set -o pipefail
mkdir -p gpurun_out/sp && export TMPDIR=/tmp
timeout -k 10 120 python tools/safeprime_probe.py > gpurun_out/sp/probe.txt 2>&1 || { tail gpurun_out/sp/probe.txt; exit 1; }
cat gpurun_out/sp/probe.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sp/prof -o sp -- python3 tools/safeprime_probe.py > gpurun_out/sp/probe_prof.txt 2>&1 || exit 1
find gpurun_out/sp/prof -name '*kernel_stats*' -exec cat {} \;
