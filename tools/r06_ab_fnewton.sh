#!/bin/bash
# A/B of the fused Newton step (MJW_FUSED_NEWTON=1) against the two-kernel Newton path, same box; the CG
# lines of the counter-reset kernel; then the sparse J'f column probe (tools/r06_jt_probe.py).
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
line() {
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(round(d['value']/1e6,3),'M', round(d['ms_per_step'],4), {k.split('<')[0].split('::')[-1]+('<'+k.split('<')[1][:12] if '<' in k else ''): round(v['ms_per_step'],4) for k,v in d['roofline']['kernels'].items()})" "$1"
}
timeout -k 10 300 python -u -m pytest tests/test_api.py tests/test_fused_paths.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_fn_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r06_fn_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  while IFS= read -r args; do
    [ -z "$args" ] && continue
    for f in 0 1; do
      MJW_FUSED_NEWTON=$f timeout -k 10 300 python -u bench.py $args --cpu-baseline 0 < /dev/null > gpurun_out/ab_fn.log 2>&1 || { tail -3 gpurun_out/ab_fn.log; exit 1; }
      echo "rep $rep fusedNewton=$f [$args]: $(line gpurun_out/ab_fn.log)"
    done
  done <<LIST
--steps 20 --warmup 5 --solver NEWTON
--steps 300 --warmup 20 --solver NEWTON
--steps 20 --warmup 5
--steps 300 --warmup 20
LIST
done
timeout -k 10 300 python -u tools/r06_jt_probe.py aloha_cloth 64 25 < /dev/null > gpurun_out/r06_jt_probe.log 2>&1; cat gpurun_out/r06_jt_probe.log | tail -30
exit 0
