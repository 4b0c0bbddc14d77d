#!/bin/bash
# round-5 A/B on the humanoid driver window (bench.py --steps 20 --warmup 5): default build against the
# dense kernel at 4 waves / SIMD (libmjw_amd_wpe4.so) and the last commit
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for r in 1 2 3; do
MODEL=humanoid timeout -k 10 600 bash tools/ab_libenv.sh 20 "-|" "mujoco_warp_amd/libmjw_amd_wpe4.so|" "mujoco_warp_amd/libmjw_amd_head.so|" || exit 1
done
MODEL=humanoid timeout -k 10 600 bash tools/ab_libenv.sh 200 "-|" "mujoco_warp_amd/libmjw_amd_wpe4.so|" || exit 1
