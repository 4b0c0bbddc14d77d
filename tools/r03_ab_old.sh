#!/bin/bash
# same-box A/B of the current tree against an older build kept in _ab_old/ (a git worktree of an earlier
# commit, built in place): alternating short humanoid bench lines
export TMPDIR=/tmp; mkdir -p gpurun_out
R=$(pwd)
line() {
  python3 -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);r=d['roofline'];print('$2', round(d['value']), round(d['ms_per_step'],4), {k: round(v['ms_per_step'],4) for k,v in r['kernels'].items()})"
}
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --cpu-baseline 0 --steps 1000 "$@" > gpurun_out/r03_abo_new$i.log 2>&1 || exit 1
  line gpurun_out/r03_abo_new$i.log new$i
  (cd _ab_old && timeout -k 10 200 python3 -u bench.py --cpu-baseline 0 --steps 1000 "$@" > $R/gpurun_out/r03_abo_old$i.log 2>&1) || exit 1
  line gpurun_out/r03_abo_old$i.log old$i
done
