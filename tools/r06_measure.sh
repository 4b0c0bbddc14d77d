#!/bin/bash
# Round 6 GPU call: the -m gpu suite, the phase split of the fused humanoid step (MJW_PROFILE build,
# s_memtime marks, the driver window: 5 warm-up + 20 steps), the PMC / SQ passes of the driver's command
# (tools/profile_model.sh -> pmc_humanoid_r06.json) and the default bench line.
# usage: bash tools/r06_measure.sh [tests|prof|pmc|bench]...   (default: all, in that order)
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
steps=${*:-tests prof pmc bench}
for s in $steps; do
  case $s in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rs > gpurun_out/r06_gpu_tests.log 2>&1
      rc=$?; tail -5 gpurun_out/r06_gpu_tests.log; [ $rc -eq 0 ] || exit $rc ;;
    prof)
      timeout -k 10 300 python -u tools/phase_prof.py 8192 20 CG humanoid 5 > gpurun_out/r06_phase_humanoid.log 2>&1 || { tail -5 gpurun_out/r06_phase_humanoid.log; exit 1; }
      cat gpurun_out/r06_phase_humanoid.log ;;
    nprof)
      timeout -k 10 300 python -u tools/phase_prof.py 8192 20 NEWTON humanoid 5 > gpurun_out/r06_phase_humanoid_newton.log 2>&1 || { tail -5 gpurun_out/r06_phase_humanoid_newton.log; exit 1; }
      cat gpurun_out/r06_phase_humanoid_newton.log ;;
    sprof)
      timeout -k 10 300 python -u tools/sparse_prof.py aloha_cloth 1024 5 20 > gpurun_out/r06_sparse_prof_aloha_cloth.log 2>&1 || { tail -5 gpurun_out/r06_sparse_prof_aloha_cloth.log; exit 1; }
      cat gpurun_out/r06_sparse_prof_aloha_cloth.log ;;
    pmc)
      ROUND=r06 timeout -k 10 900 bash tools/profile_model.sh humanoid > gpurun_out/prof_humanoid.log 2>&1 || { tail -5 gpurun_out/prof_humanoid.log; exit 1; }
      cp gpurun_out/pmc_humanoid_r06.json profiles/ || exit 1
      cat gpurun_out/r06_humanoid_sq_counters.txt | grep -A12 step_kernel ;;
    bench)
      timeout -k 10 400 python3 -u bench.py > gpurun_out/r06_bench_humanoid.log 2>&1 || { tail -5 gpurun_out/r06_bench_humanoid.log; exit 1; }
      tail -1 gpurun_out/r06_bench_humanoid.log | cut -c1-400 ;;
  esac
done
exit 0
