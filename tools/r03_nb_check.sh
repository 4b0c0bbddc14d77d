export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_primitives.py tests/test_gpu_parity_strict.py tests/test_franka_boxes.py tests/test_ccd.py tests/test_gpu_parity_models.py tests/test_api.py tests/test_tendon.py tests/test_elliptic.py tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r03_nb_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r03_nb_tests.log
[ $rc -eq 0 ] || exit $rc
for mdl in franka humanoid apollo; do
  timeout -k 10 200 python -u bench.py --model $mdl --cpu-baseline 0 --steps 500 > gpurun_out/r03_nb_bench_$mdl.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r03_nb_bench_$mdl.log').read().splitlines()[-1]);r=d['roofline'];print('$mdl', round(d['value']), round(d['ms_per_step'],4), {k: round(v['ms_per_step'],4) for k,v in r['kernels'].items()})"
done
