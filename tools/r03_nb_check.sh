#!/bin/bash
# round-3 check of the factor-bound / world-order changes: affected GPU tests, then short bench lines
# (franka, apollo, humanoid with the forward order on and off)
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_primitives.py tests/test_gpu_parity_strict.py tests/test_franka_boxes.py tests/test_ccd.py tests/test_gpu_parity_models.py tests/test_api.py tests/test_tendon.py tests/test_elliptic.py tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r03_nb_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r03_nb_tests.log
[ $rc -eq 0 ] || exit $rc
line() {
  python3 -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);r=d['roofline'];print('$2', round(d['value']), round(d['ms_per_step'],4), {k: round(v['ms_per_step'],4) for k,v in r['kernels'].items()})"
}
for mdl in franka apollo humanoid; do
  timeout -k 10 200 python -u bench.py --model $mdl --cpu-baseline 0 --steps 500 > gpurun_out/r03_nb_bench_$mdl.log 2>&1 || exit 1
  line gpurun_out/r03_nb_bench_$mdl.log $mdl
done
MJW_FWD_ORDER=0 timeout -k 10 200 python -u bench.py --cpu-baseline 0 --steps 500 > gpurun_out/r03_nb_bench_humanoid_nofwd.log 2>&1 || exit 1
line gpurun_out/r03_nb_bench_humanoid_nofwd.log humanoid_nofwd
timeout -k 10 200 python -u bench.py --cpu-baseline 0 --steps 500 > gpurun_out/r03_nb_bench_humanoid2.log 2>&1 || exit 1
line gpurun_out/r03_nb_bench_humanoid2.log humanoid_fwd2
