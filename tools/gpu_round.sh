#!/bin/bash
# GPU check used with gpurun: parity tests, short bench, stage timings.
# Stops at the first GPU fault / abort / timeout (exit codes other than 0 and pytest's 1).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
STEPS=${STEPS:-300}
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/parity.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/parity.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps "$STEPS" --cpu-baseline 0 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
timeout -k 10 300 python tools/stage_times.py 8192 100 ${SOLVER:-CG} > gpurun_out/stages.log 2>&1 || exit $?
tail -1 gpurun_out/stages.log
if [ -f mujoco_warp_amd/libmjw_amd_prof.so ]; then
  timeout -k 10 300 python tools/phase_prof.py 8192 100 ${SOLVER:-CG} > gpurun_out/phase.json 2>&1 || exit $?
  cat gpurun_out/phase.json
fi
exit $rc
