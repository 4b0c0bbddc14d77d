#!/bin/bash
# Round 5 end-of-round measurement, part B: the bench lines of the other configs (C3 franka, C4 apollo,
# C5 aloha_cloth, the reference's cloth benchmark, humanoid with its default Newton solver, and the
# humanoid 1000-step line).
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "franka|--model franka" "apollo|--model apollo" "cloth|--model cloth" "aloha_cloth|--model aloha_cloth" "humanoid_newton|--solver NEWTON" "humanoid_1000|--steps 1000 --warmup 20"; do
  tag=${spec%%|*}; args=${spec#*|}
  timeout -k 10 400 python3 -u bench.py $args --cpu-baseline 0 > gpurun_out/bench_$tag.log 2>&1 || { tail -5 gpurun_out/bench_$tag.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/bench_$tag.log').read().splitlines()[-1]);r=d['roofline'];print('$tag', round(d['value'],1), 'ms/step', round(d['ms_per_step'],4), r['group'], round(r['kernel_ms'],4), 'frac', round(r['frac'],4))"
done
