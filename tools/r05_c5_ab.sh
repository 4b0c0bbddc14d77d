#!/bin/bash
# C5 collision-item A/B: aloha_cloth base / new / split-off, then the flex parity tests on the default build
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
MODEL=aloha_cloth bash tools/ab_libenv.sh 30 "mujoco_warp_amd/libmjw_amd_base.so|X=0" "-|X=0" "mujoco_warp_amd/libmjw_amd_v0.so|X=0" "mujoco_warp_amd/libmjw_amd_base.so|X=0" "-|X=0" || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_cloth.py tests/test_flex_dims.py tests/test_gpu_golden.py > gpurun_out/c5ab_tests.log 2>&1 || { tail -30 gpurun_out/c5ab_tests.log; exit 1; }
tail -2 gpurun_out/c5ab_tests.log
