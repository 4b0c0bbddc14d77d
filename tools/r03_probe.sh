#!/bin/bash
# round-3 probe: world-order A/B (bench lines with the launch trace; lean per-wave lifetimes), C3-C5 parity report, GPU tests
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for tag in on off on2 off2; do
  case $tag in off*) export MJW_WORLD_ORDER=0;; *) export MJW_WORLD_ORDER=1;; esac
  timeout -k 10 300 python -u bench.py --steps 300 --cpu-baseline 0 > gpurun_out/r03_probe_bench_$tag.log 2>&1 || exit $?
  tail -1 gpurun_out/r03_probe_bench_$tag.log | cut -c1-200
done
export MJW_WORLD_ORDER=1
timeout -k 10 300 python -u tools/wave_log.py 8192 50 CG gpurun_out/r03_wave_log_cg.json > gpurun_out/r03_wave_log.log 2>&1 || exit $?
MJW_WORLD_ORDER=0 timeout -k 10 300 python -u tools/wave_log.py 8192 50 CG gpurun_out/r03_wave_log_cg_noorder.json >> gpurun_out/r03_wave_log.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/parity_models.py gpurun_out/r03_parity_models.json > gpurun_out/r03_parity_models.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_probe_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03_probe_tests.log; exit $rc
