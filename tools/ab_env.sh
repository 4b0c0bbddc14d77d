#!/bin/bash
# A/B of environment settings on the headline bench: bash tools/ab_env.sh STEPS "ENV=1" "ENV=2" ...
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
STEPS=$1; shift
MODEL=${MODEL:-humanoid}
i=0
for setting in "$@"; do
  env $setting timeout -k 10 200 python -u bench.py --model $MODEL --steps $STEPS --cpu-baseline 0 > gpurun_out/abenv_$i.log 2>&1 || exit $?
  echo "$setting: $(python3 -c "import json;d=json.loads(open('gpurun_out/abenv_$i.log').read().splitlines()[-1]);r=d['roofline'];print(round(d['value']/1e6,3),'M', 'ms/step', round(d['ms_per_step'],4), 'fwd', round(r['kernel_ms'],4), 'dense', round(list(r['other_kernels'].values())[0]['ms'],4), 'frac', round(r['frac'],4))")"
  i=$((i+1))
done
