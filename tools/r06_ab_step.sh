#!/bin/bash
# Same-box A/B of step-kernel library variants (tools/build_variants.py mjw_step.hip ...): the world-order
# tests on the first variant, then humanoid CG (driver window, 300 steps), Newton and franka lines per variant.
# usage: bash tools/r06_ab_step.sh name1 name2 ...  ("-" = libmjw_amd.so)
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
lp() { if [ "$1" = "-" ]; then echo ""; else echo "MJW_LIB_PATH=$PWD/mujoco_warp_amd/libmjw_amd_$1.so"; fi; }
env $(lp $1) timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_api.py tests/test_fused_paths.py} -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_abs_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r06_abs_tests.log; [ $rc -eq 0 ] || exit $rc
line() {
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(round(d['value']/1e6,3),'M', round(d['ms_per_step'],4), {k.split('::')[-1][:22]: round(v['ms_per_step'],4) for k,v in d['roofline']['kernels'].items()})" "$1"
}
for rep in 1 2; do
  for v in "$@"; do
    while IFS= read -r args; do
      [ -z "$args" ] && continue
      env $(lp $v) timeout -k 10 300 python -u bench.py $args --cpu-baseline 0 < /dev/null > gpurun_out/abs.log 2>&1 || { tail -3 gpurun_out/abs.log; exit 1; }
      echo "rep $rep $v [$args]: $(line gpurun_out/abs.log)"
    done <<LIST
--steps 20 --warmup 5
--steps 300 --warmup 20
--steps 300 --warmup 20 --solver NEWTON
--model franka --steps 300 --warmup 20
LIST
  done
done
exit 0
