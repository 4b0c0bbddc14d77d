#!/bin/bash
# GPU check of a build: the -m gpu suite, then the humanoid bench lines (driver window, 300 steps, Newton).
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rs > gpurun_out/r06_gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r06_gpu_tests.log; grep FAILED gpurun_out/r06_gpu_tests.log | head -20; [ $rc -eq 0 ] || exit $rc
for args in "--steps 20 --warmup 5" "--steps 300 --warmup 20" "--steps 300 --warmup 20 --solver NEWTON"; do
  timeout -k 10 300 python -u bench.py $args --cpu-baseline 0 > gpurun_out/chk.log 2>&1 || { tail -3 gpurun_out/chk.log; exit 1; }
  echo "[$args] $(python3 -c "import json;d=json.loads(open('gpurun_out/chk.log').read().splitlines()[-1]);print(round(d['value']/1e6,3),'M', round(d['ms_per_step'],4), {k: round(v['ms_per_step'],4) for k,v in d['roofline']['kernels'].items()})")"
done
