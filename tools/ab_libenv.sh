#!/bin/bash
# A/B over (library, env) pairs: bash tools/ab_libenv.sh STEPS "lib.so|ENV=1" ...  (lib "-" = default build)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
STEPS=$1; shift
MODEL=${MODEL:-humanoid}
EXTRA=${EXTRA:-}  # extra bench.py arguments, e.g. "--solver NEWTON"
i=0
for spec in "$@"; do
  lib=${spec%%|*}; envs=${spec#*|}
  if [ "$lib" = "-" ]; then lp=""; else lp="MJW_LIB_PATH=$PWD/$lib"; fi
  env $lp $envs timeout -k 10 300 python -u bench.py --model $MODEL --steps $STEPS --cpu-baseline 0 $EXTRA > gpurun_out/ablib_$i.log 2>&1 || exit $?
  echo "$spec: $(python3 -c "import json;d=json.loads(open('gpurun_out/ablib_$i.log').read().splitlines()[-1]);print(round(d['value']/1e3,2),'K', round(d['ms_per_step'],4), {k: round(v['ms_per_step'],4) for k,v in d['roofline']['kernels'].items()})")"
  i=$((i+1))
done
