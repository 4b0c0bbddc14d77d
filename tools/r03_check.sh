#!/bin/bash
# round-3 check: full GPU test suite (no -x), C3-C5 parity report, sparse light probe
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r03_check_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r03_check_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u tools/parity_models.py gpurun_out/r03_parity_models.json > gpurun_out/r03_parity_models.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/light_probe.py > gpurun_out/r03_light_probe.log 2>&1 || exit $?
exit $rc
