#!/bin/bash
# End-of-round measurement on one GPU (round 4): rocprofv3 kernel stats + PMC traffic + SQ counters of the
# given configs (tools/profile_model.sh), their PMC summaries copied into profiles/ so that bench.py binds
# them, then the bench line of every config into gpurun_out/bench_<tag>.log.  Stops at the first failure.
# usage: bash tools/r04_measure.sh "humanoid aloha_cloth" "humanoid humanoid:NEWTON franka apollo cloth aloha_cloth"
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp ROUND=${ROUND:-r04}
mkdir -p gpurun_out
for spec in $1; do
  mdl=${spec%%:*}; sol=""; [ "$spec" != "$mdl" ] && sol=${spec#*:}
  bash tools/profile_model.sh $mdl $sol || exit $?
  tag=$mdl; [ -n "$sol" ] && tag=${mdl}_$(echo $sol | tr 'A-Z' 'a-z')
  cp gpurun_out/pmc_${tag}_${ROUND}.json profiles/ || exit 1
done
for spec in $2; do
  mdl=${spec%%:*}; sol=""; [ "$spec" != "$mdl" ] && sol=${spec#*:}
  tag=$mdl; args="--model $mdl"; [ -n "$sol" ] && { tag=${mdl}_$(echo $sol | tr 'A-Z' 'a-z'); args="$args --solver $sol"; }
  cpu="--cpu-baseline 0"; [ "$tag" = humanoid ] && cpu=""
  timeout -k 10 400 python3 -u bench.py $args $cpu > gpurun_out/bench_$tag.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads(open('gpurun_out/bench_$tag.log').read().splitlines()[-1]);r=d['roofline'];print('$tag', round(d['value'],1), 'ms/step', round(d['ms_per_step'],4), 'kernel', r['kernel'], 'kernel_ms', round(r['kernel_ms'],4), 'frac', round(r['frac'],4), 'traffic', r['traffic'], 'cpu', (d['cpu_baseline'] or {}).get('value'))"
done
exit 0
