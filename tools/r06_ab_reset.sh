#!/bin/bash
# Same-box probe of the counter-reset kernel's cost: library variants, humanoid CG driver window and 300 steps.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for v in "$@"; do
    for args in "--steps 20 --warmup 5" "--steps 300 --warmup 20"; do
      MJW_LIB_PATH=$PWD/mujoco_warp_amd/libmjw_amd_$v.so timeout -k 10 300 python -u bench.py $args --cpu-baseline 0 < /dev/null > gpurun_out/abr.log 2>&1 || { tail -3 gpurun_out/abr.log; exit 1; }
      echo "rep $rep $v [$args]: $(python3 -c "import json,sys;d=json.loads(open('gpurun_out/abr.log').read().splitlines()[-1]);print(round(d['value']/1e6,3),'M', round(d['ms_per_step'],4), {k.split('::')[-1][:22]: round(v['ms_per_step'],4) for k,v in d['roofline']['kernels'].items()})")"
    done
  done
done
exit 0
