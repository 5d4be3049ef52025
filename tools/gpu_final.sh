# round-end validation: GPU suite + smoke, default bench line, kernel-trace stats of the bench command -> gpurun_out/$1
set -o pipefail
O=gpurun_out/${1:-final}
bash tools/gpu_suite.sh ${1:-final} && bash tools/gpu_bench_prof.sh ${1:-final}
