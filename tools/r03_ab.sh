#!/bin/bash
# A/B bench lines (round 3): env settings x models, short runs, kernel times per step
export TMPDIR=/tmp; mkdir -p gpurun_out
line() {
  python3 -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);r=d['roofline'];print('$2', round(d['value']), round(d['ms_per_step'],4), {k: round(v['ms_per_step'],4) for k,v in r['kernels'].items()})"
}
i=0
for spec in "$@"; do   # spec: model[:ENV=VAL[,ENV=VAL]]
  mdl=${spec%%:*}; envs=""
  [ "$mdl" != "$spec" ] && envs=$(echo "${spec#*:}" | tr ',' ' ')
  i=$((i+1))
  env $envs timeout -k 10 200 python3 -u bench.py --model $mdl --cpu-baseline 0 --steps 500 > gpurun_out/r03_ab_$i.log 2>&1 || exit 1
  line gpurun_out/r03_ab_$i.log "$spec"
done
