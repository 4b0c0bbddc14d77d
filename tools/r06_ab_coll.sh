#!/bin/bash
# A/B of the sparse collision launch (sp::forward_kernel<1024>) without dynamically indexed stack arrays
# (round 6) against the library before it (libmjw_amd_base.so), aloha_cloth and cloth, interleaved; then
# the sparse / flex / collision GPU tests on the new library.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in mujoco_warp_amd/libmjw_amd_base.so -; do
    lp=""; [ "$lib" != "-" ] && lp="MJW_LIB_PATH=$PWD/$lib"
    for model in aloha_cloth cloth; do
      env $lp timeout -k 10 300 python -u bench.py --model $model --steps 20 --warmup 20 --cpu-baseline 0 > gpurun_out/abcoll.log 2>&1 || exit $?
      echo "rep $rep $lib $model: $(python3 -c "import json;d=json.loads(open('gpurun_out/abcoll.log').read().splitlines()[-1]);print(round(d['value']/1e3,2),'K', round(d['ms_per_step'],3), {k.split('(')[0]: round(v['ms_per_step'],3) for k,v in d['roofline']['kernels'].items() if v['ms_per_step'] > 0.05})")"
    done
  done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "cloth or flex or golden or mesh or sparse or collision or hfield or tactile" > gpurun_out/r06_coll_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r06_coll_tests.log; exit $rc
