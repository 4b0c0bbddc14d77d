#!/bin/bash
# round-3 probe: new bench line (launch trace), per-wave lifetimes of both kernels, kernel stats
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 300 --cpu-baseline 0 > gpurun_out/r03_probe_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r03_probe_bench.log
timeout -k 10 300 python -u tools/wave_log.py 8192 50 CG gpurun_out/r03_wave_log_cg.json > gpurun_out/r03_wave_log.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/wave_log.py 8192 50 NEWTON gpurun_out/r03_wave_log_newton.json >> gpurun_out/r03_wave_log.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/phase_prof.py 8192 50 CG > gpurun_out/r03_phase_cg.json 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_bench_launch.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_probe_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/parity_models.py gpurun_out/r03_parity_models.json > gpurun_out/r03_parity_models.log 2>&1 || exit $?
exit 0
