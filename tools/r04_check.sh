#!/bin/bash
# GPU check of the round-4 tree: the whole -m gpu suite, then the driver-style bench line (20 steps) and
# a 1000-step line.  Stops at the first GPU fault / abort / timeout.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=15 -v --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -n "$NOBENCH" ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/bench20.log 2>&1 || exit $?
tail -1 gpurun_out/bench20.log | cut -c1-400
timeout -k 10 300 python -u bench.py --steps 1000 --cpu-baseline 0 > gpurun_out/bench1000.log 2>&1 || exit $?
tail -1 gpurun_out/bench1000.log | cut -c1-400
exit $rc
