#!/bin/bash
# Round 6: sparse-path GPU tests, then aloha_cloth / cloth bench lines and the sparse CG sub-phase split.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
line() {
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(round(d['value']/1e3,2),'K', round(d['ms_per_step'],3), {k.split('::')[-1][:28]: round(v['ms_per_step'],3) for k,v in d['roofline']['kernels'].items()})" "$1"
}
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_cloth.py tests/test_gpu_parity_models.py tests/test_sparse_features.py tests/test_sparse_implicit.py tests/test_flex_dims.py tests/test_unroll.py tests/test_ls_parallel.py} -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_sparse_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r06_sparse_tests.log; grep -E "FAILED|Error" gpurun_out/r06_sparse_tests.log | head; [ $rc -eq 0 ] || exit $rc
for model in aloha_cloth cloth; do
  timeout -k 10 300 python -u bench.py --model $model --cpu-baseline 0 < /dev/null > gpurun_out/sc_b.log 2>&1 || { tail -3 gpurun_out/sc_b.log; exit 1; }
  echo "[$model]: $(line gpurun_out/sc_b.log)"
done
if [ "${PROF:-1}" = 1 ]; then
  timeout -k 10 300 python -u tools/sparse_prof.py aloha_cloth 1024 5 20 < /dev/null > gpurun_out/r06_sparse_prof3.log 2>&1 || { tail -5 gpurun_out/r06_sparse_prof3.log; exit 1; }
  tail -18 gpurun_out/r06_sparse_prof3.log
fi
exit 0
