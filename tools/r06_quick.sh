#!/bin/bash
# Round 6 quick GPU check of a build: the named GPU test files (default: primitives, api, dense-path
# parity), then bench lines of the dense-path configs and, with PROF=1, the Newton phase split.
# usage: bash tools/r06_quick.sh [test files...]
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
tests=${*:-tests/test_gpu_primitives.py tests/test_api.py tests/test_gpu_parity_strict.py tests/test_gpu_parity_models.py tests/test_elliptic.py tests/test_fused_paths.py}
timeout -k 10 500 python -u -m pytest $tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -rs > gpurun_out/r06_quick_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r06_quick_tests.log; grep -E "FAILED|Error" gpurun_out/r06_quick_tests.log | head -20; [ $rc -eq 0 ] || exit $rc
line() {
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(round(d['value']/1e6,3),'M', round(d['ms_per_step'],4), {k.split('<')[0].split('::')[-1]+('<'+k.split('<')[1][:12] if '<' in k else ''): round(v['ms_per_step'],4) for k,v in d['roofline']['kernels'].items()})" "$1"
}
while IFS= read -r args; do
  [ -z "$args" ] && continue
  timeout -k 10 300 python -u bench.py $args --cpu-baseline 0 < /dev/null > gpurun_out/quick_bench.log 2>&1 || { tail -3 gpurun_out/quick_bench.log; exit 1; }
  echo "[$args]: $(line gpurun_out/quick_bench.log)"
done <<EOF
--steps 20 --warmup 5
--steps 300 --warmup 20
--steps 300 --warmup 20 --solver NEWTON
--model franka --steps 300 --warmup 20
--model apollo --steps 300 --warmup 20
EOF
if [ "${PROF:-0}" = 1 ]; then
  timeout -k 10 300 python -u tools/phase_prof.py 8192 20 NEWTON humanoid 5 > gpurun_out/r06_phase_newton.log 2>&1 || { tail -5 gpurun_out/r06_phase_newton.log; exit 1; }
  cat gpurun_out/r06_phase_newton.log
fi
exit 0
