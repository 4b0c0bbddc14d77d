#!/bin/bash
# End-of-round measurement on one GPU: rocprof passes (humanoid, aloha_cloth), then the bench line of
# every config into gpurun_out/bench_<model>.log.  Stops at the first failing step.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_profile.sh || exit $?
bash tools/gpu_profile_sparse.sh aloha_cloth || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/bench_humanoid.log 2>&1 || exit $?
for mdl in franka apollo cloth; do
  timeout -k 10 300 python -u bench.py --model $mdl --cpu-baseline 0 > gpurun_out/bench_$mdl.log 2>&1 || exit $?
done
timeout -k 10 300 python -u bench.py --model aloha_cloth > gpurun_out/bench_aloha_cloth.log 2>&1 || exit $?
for mdl in humanoid franka apollo cloth aloha_cloth; do
  python3 -c "import json;d=json.loads(open('gpurun_out/bench_$mdl.log').read().splitlines()[-1]);r=d['roofline'];print('$mdl', round(d['value'],1), 'ms/step', round(d['ms_per_step'],4), 'kernel_ms', round(r['kernel_ms'],4), 'frac', round(r['frac'],4), 'traffic', r['traffic'], 'cpu', (d['cpu_baseline'] or {}).get('value'))"
done
