#!/bin/bash
# round-5 A/B: the fused whole-step kernel (default) against the forward + dense kernels (MJW_FUSED=0),
# humanoid CG (driver window, 1000 steps) and Newton; the dense-path parity tests first
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_parity_strict.py tests/test_graph.py tests/test_ls_parallel.py tests/test_elliptic.py > gpurun_out/ab3_tests.log 2>&1 || { tail -15 gpurun_out/ab3_tests.log; exit 1; }
tail -2 gpurun_out/ab3_tests.log
for r in 1 2; do
MODEL=humanoid timeout -k 10 600 bash tools/ab_libenv.sh 20 "-|" "-|MJW_FUSED=0" || exit 1
done
MODEL=humanoid timeout -k 10 600 bash tools/ab_libenv.sh 200 "-|" "-|MJW_FUSED=0" || exit 1
