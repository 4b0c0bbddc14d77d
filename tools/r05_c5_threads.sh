#!/bin/bash
# C5 CG launch: 256 (default) vs 512 / 1024 threads per world (MJW_SP_SOLVE_THREADS variant builds)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for M in aloha_cloth cloth; do
  MODEL=$M bash tools/ab_libenv.sh 30 "-|X=0" "mujoco_warp_amd/libmjw_amd_t512.so|X=0" "mujoco_warp_amd/libmjw_amd_t1024.so|X=0" "-|X=0" "mujoco_warp_amd/libmjw_amd_t512.so|X=0" || exit 1
done
