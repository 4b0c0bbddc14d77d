#!/bin/bash
# The driver's headline command (bench.py --steps 20 --warmup 5) run 5 times back to back: run-to-run spread
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for i in 1 2 3 4 5; do
  timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/rep_$i.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads([l for l in open('gpurun_out/rep_$i.log') if l.startswith('{')][-1]);print('run $i', round(d['value']/1e6,3), 'M env-steps/s', round(d['ms_per_step'],4), 'ms/step', 'niter', round(d['config']['solver_niter_mean'],2))"
done
