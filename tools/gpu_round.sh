#!/bin/bash
# GPU check used with gpurun: parity tests, short bench, rocprof kernel stats of the bench.
# Stops at the first GPU fault / abort / timeout (exit codes other than 0 and pytest's 1).
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-300}
TAG=${TAG:-r02}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/parity.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/parity.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps "$STEPS" --cpu-baseline 0 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 50 --cpu-baseline 0 > gpurun_out/prof_$TAG.log 2>&1 || exit $?
exit $rc
