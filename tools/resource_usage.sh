#!/bin/bash
# VGPR / SGPR / scratch / occupancy of every kernel in one translation unit (hipcc -Rpass-analysis).
# usage: bash tools/resource_usage.sh mujoco_warp_amd/csrc/mjw_step.hip [kernel-substring]
cd "$(dirname "$0")/.." || exit 1
src=$1; pat=${2:-}
hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=on -I include -c "$src" -o /tmp/ru.o -Rpass-analysis=kernel-resource-usage 2>&1 \
  | grep -E "Function Name|VGPRs:|AGPRs|ScratchSize|Occupancy|LDS Size" | sed 's/.*remark: //' \
  | awk -v pat="$pat" '/Function Name/{show = (pat == "" || index($0, pat) > 0)} show'
