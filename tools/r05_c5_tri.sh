#!/bin/bash
# C5 collision launch: flex-triangle candidates at compile-time slots (variant build) vs the default
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
MODEL=aloha_cloth bash tools/ab_libenv.sh 30 "-|X=0" "mujoco_warp_amd/libmjw_amd_tri.so|X=0" "-|X=0" "mujoco_warp_amd/libmjw_amd_tri.so|X=0"
