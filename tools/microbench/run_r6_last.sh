# last measurements of the round-6 tree: default bench + config-2 kernel trace, then the PMC passes
set -o pipefail
bash tools/microbench/run_r6_final.sh final6 && bash tools/microbench/run_r6_pmc.sh
