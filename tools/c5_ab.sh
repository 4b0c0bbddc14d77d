#!/bin/bash
# sparse-path GPU tests, then the C5 / cloth bench with and without the LDS-resident solve
cd "$(dirname "$0")/.." || exit 1
timeout -k 10 500 python -u -m pytest tests/test_cloth.py tests/test_mesh.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/c5tests.log 2>&1; rc=$?; tail -3 gpurun_out/c5tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
MODEL=aloha_cloth bash tools/ab_env.sh 50 "MJW_SP_SOLVE_LDS=1" "MJW_SP_SOLVE_LDS=0" || exit $?
MODEL=cloth bash tools/ab_env.sh 100 "MJW_SP_SOLVE_LDS=1" "MJW_SP_SOLVE_LDS=0" || exit $?
exit $rc
