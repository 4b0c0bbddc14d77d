#!/bin/bash
# Round 6 final GPU call: the whole -m gpu suite, the rocprofv3 passes of the headline (driver window:
# pmc_humanoid_r06.json, SQ counters, kernel stats) and of aloha_cloth, then the default bench line (which
# prices the new PMC summary) and the driver-window line.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rs > gpurun_out/r06_gpu_tests.log 2>&1
  rc=$?; tail -4 gpurun_out/r06_gpu_tests.log; grep FAILED gpurun_out/r06_gpu_tests.log | head -20; [ $rc -eq 0 ] || exit $rc
fi
# MODELS entries: model or model:SOLVER (e.g. humanoid:NEWTON -> pmc_humanoid_newton_r06.json)
for spec in ${MODELS:-humanoid aloha_cloth}; do
  mdl=${spec%%:*}; sol=""; tag=$mdl
  if [ "$spec" != "$mdl" ]; then sol=${spec#*:}; tag=${mdl}_$(echo "$sol" | tr 'A-Z' 'a-z'); fi
  ROUND=r06 timeout -k 10 900 bash tools/profile_model.sh $mdl $sol > gpurun_out/prof_$tag.log 2>&1 || { tail -5 gpurun_out/prof_$tag.log; exit 1; }
  cp gpurun_out/pmc_${tag}_r06.json profiles/ || exit 1
  tail -1 gpurun_out/prof_$tag.log
done
timeout -k 10 400 python3 -u bench.py < /dev/null > gpurun_out/r06_bench_humanoid.log 2>&1 || { tail -5 gpurun_out/r06_bench_humanoid.log; exit 1; }
tail -1 gpurun_out/r06_bench_humanoid.log | cut -c1-300
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 < /dev/null > gpurun_out/r06_bench_driver.log 2>&1 || { tail -5 gpurun_out/r06_bench_driver.log; exit 1; }
tail -1 gpurun_out/r06_bench_driver.log | cut -c1-300
exit 0
