#!/bin/bash
# A/B of fp32 division / sqrt codegen: the default (correctly rounded) library against one built with
# -fno-hip-fp32-correctly-rounded-divide-sqrt (libmjw_amd_nodiv.so), interleaved, same box; humanoid CG
# on the driver's window and 300 steps, then the Newton and franka configs.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for rep in 1 2 3; do
  for lib in - mujoco_warp_amd/libmjw_amd_nodiv.so; do
    lp=""; [ "$lib" != "-" ] && lp="MJW_LIB_PATH=$PWD/$lib"
    env $lp timeout -k 10 200 python -u bench.py --steps 300 --warmup 20 --cpu-baseline 0 > gpurun_out/abdiv.log 2>&1 || exit $?
    echo "rep $rep $lib humanoid300: $(python3 -c "import json;d=json.loads(open('gpurun_out/abdiv.log').read().splitlines()[-1]);print(round(d['value']/1e6,3),'M', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4))")"
  done
done
for lib in - mujoco_warp_amd/libmjw_amd_nodiv.so; do
  lp=""; [ "$lib" != "-" ] && lp="MJW_LIB_PATH=$PWD/$lib"
  for cfg in "--solver NEWTON" "--model franka" "--model apollo"; do
    env $lp timeout -k 10 200 python -u bench.py --steps 300 --warmup 20 --cpu-baseline 0 $cfg > gpurun_out/abdiv.log 2>&1 || exit $?
    echo "$lib [$cfg]: $(python3 -c "import json;d=json.loads(open('gpurun_out/abdiv.log').read().splitlines()[-1]);print(round(d['value']/1e6,3),'M', round(d['ms_per_step'],4))")"
  done
done
