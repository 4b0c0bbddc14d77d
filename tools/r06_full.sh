#!/bin/bash
# Round 6 full check: the whole -m gpu suite, then a bench line per config (driver window for humanoid).
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rs > gpurun_out/r06_gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r06_gpu_tests.log; grep FAILED gpurun_out/r06_gpu_tests.log | head -20; [ $rc -eq 0 ] || exit $rc
line() {
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(round(d['value']/1e6,4),'M', round(d['ms_per_step'],4), {k.split('::')[-1][:30]: round(v['ms_per_step'],4) for k,v in d['roofline']['kernels'].items()})" "$1"
}
while IFS= read -r args; do
  [ -z "$args" ] && continue
  timeout -k 10 300 python -u bench.py $args --cpu-baseline 0 < /dev/null > gpurun_out/full_b.log 2>&1 || { tail -3 gpurun_out/full_b.log; exit 1; }
  echo "[$args]: $(line gpurun_out/full_b.log)"
done <<LIST
--steps 20 --warmup 5
--steps 1000 --warmup 20
--steps 1000 --warmup 20 --solver NEWTON
--model franka
--model apollo
--model aloha_cloth
--model cloth
LIST
exit 0
