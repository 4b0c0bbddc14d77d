#!/bin/bash
# Same-box A/B of dense-kernel library variants: humanoid Newton, apollo, franka lines, two rounds.
# usage: bash tools/r06_ab_dense.sh name1 name2 ...
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
line() {
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(round(d['value']/1e6,3),'M', round(d['ms_per_step'],4), {k.split('::')[-1][:22]: round(v['ms_per_step'],4) for k,v in d['roofline']['kernels'].items() if 'dense' in k})" "$1"
}
for rep in 1 2; do
  for v in "$@"; do
    for args in "--steps 300 --warmup 20 --solver NEWTON" "--model apollo --steps 300 --warmup 20" "--model franka --steps 300 --warmup 20"; do
      MJW_LIB_PATH=$PWD/mujoco_warp_amd/libmjw_amd_$v.so timeout -k 10 300 python -u bench.py $args --cpu-baseline 0 < /dev/null > gpurun_out/abd.log 2>&1 || { tail -3 gpurun_out/abd.log; exit 1; }
      echo "rep $rep $v [$args]: $(line gpurun_out/abd.log)"
    done
  done
done
exit 0
