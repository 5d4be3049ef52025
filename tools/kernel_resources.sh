#!/bin/bash
# VGPRs / scratch / occupancy of each k_modexp geometry (gfx950), from the compiler's resource remarks.
# usage: tools/kernel_resources.sh [geom ids...] [-- extra hipcc flags]
cd "$(dirname "$0")/.." || exit 1
ids=(); extra=()
while [ $# -gt 0 ]; do [ "$1" = "--" ] && { shift; extra=("$@"); break; }; ids+=("$1"); shift; done
[ ${#ids[@]} -eq 0 ] && ids=(0 1 2 3 4 5 6)
for g in "${ids[@]}"; do
  ( /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include --cuda-device-only -c -o /dev/null \
      -DMPCX_GEOM_ID=$g "${extra[@]}" mpcium_amd/csrc/mpcx_geom.hip -Rpass-analysis=kernel-resource-usage 2>&1 \
    | grep -E "VGPRs:|ScratchSize|Occupancy" | sed 's/.*remark: [^ ]* *//; s/ \[-Rpass.*//' | tr '\n' ' ' ; echo " <- geom $g" ) &
done
wait
