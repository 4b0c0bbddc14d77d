#!/bin/bash
# round-5 A/B: the convex pre-pass at 2 waves / SIMD and Newton dense kernels at 3 (default build) against
# the last commit (libmjw_amd_head.so) on apollo (C4) and humanoid Newton; the CCD parity tests first
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_collision_types.py tests/test_multiccd.py tests/test_hfield.py tests/test_golden.py tests/test_gpu_golden.py > gpurun_out/ab2_tests.log 2>&1 || { tail -15 gpurun_out/ab2_tests.log; exit 1; }
tail -2 gpurun_out/ab2_tests.log
for r in 1 2; do
MODEL=apollo timeout -k 10 600 bash tools/ab_libenv.sh 20 "-|" "mujoco_warp_amd/libmjw_amd_head.so|" || exit 1
done
