#!/bin/bash
# Same-box A/B of sparse-path library variants (tools/build_variants.py): aloha_cloth and cloth bench lines
# per variant, two rounds.  usage: bash tools/r06_sparse_ab.sh name1 name2 ...  ("-" = libmjw_amd.so)
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
line() {
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);k=d['roofline']['kernels'];print(round(d['value']/1e3,2),'K', round(d['ms_per_step'],3), 'solve', round(sum(v['ms_per_step'] for n,v in k.items() if 'solve_kernel' in n),3))" "$1"
}
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = "-" ]; then lp=""; else lp="MJW_LIB_PATH=$PWD/mujoco_warp_amd/libmjw_amd_$v.so"; fi
    for model in aloha_cloth cloth; do
      env $lp timeout -k 10 300 python -u bench.py --model $model --cpu-baseline 0 < /dev/null > gpurun_out/sab.log 2>&1 || { tail -3 gpurun_out/sab.log; exit 1; }
      echo "rep $rep $v $model: $(line gpurun_out/sab.log)"
    done
  done
done
exit 0
