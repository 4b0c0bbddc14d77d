#!/bin/bash
# Round 6: world-order tests + humanoid CG lines of the counter-reset kernel, then the sparse CG sub-phase
# split (profile build) and the J'f column probe on aloha_cloth.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
line() {
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(round(d['value']/1e6,3),'M', round(d['ms_per_step'],4), {k.split('<')[0].split('::')[-1]+('<'+k.split('<')[1][:12] if '<' in k else ''): round(v['ms_per_step'],4) for k,v in d['roofline']['kernels'].items()})" "$1"
}
timeout -k 10 300 python -u -m pytest tests/test_api.py tests/test_gpu_primitives.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_sp_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r06_sp_tests.log; [ $rc -eq 0 ] || exit $rc
for args in "--steps 20 --warmup 5" "--steps 20 --warmup 5" "--steps 300 --warmup 20"; do
  timeout -k 10 300 python -u bench.py $args --cpu-baseline 0 < /dev/null > gpurun_out/sp_b.log 2>&1 || { tail -3 gpurun_out/sp_b.log; exit 1; }
  echo "[$args]: $(line gpurun_out/sp_b.log)"
done
timeout -k 10 300 python -u tools/sparse_prof.py aloha_cloth 1024 5 20 < /dev/null > gpurun_out/r06_sparse_prof2.log 2>&1 || { tail -5 gpurun_out/r06_sparse_prof2.log; exit 1; }
tail -45 gpurun_out/r06_sparse_prof2.log
timeout -k 10 300 python -u tools/r06_jt_probe.py aloha_cloth 64 25 < /dev/null > gpurun_out/r06_jt_probe.log 2>&1; tail -30 gpurun_out/r06_jt_probe.log
exit 0
