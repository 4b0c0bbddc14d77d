#!/bin/bash
# Round-3 measurement on one GPU.  usage: bash tools/r03_measure.sh <config> ...
# config: humanoid | humanoid:NEWTON | franka | apollo | aloha_cloth | cloth (profile + bench line) or
# bench:<model>[:<solver>] (bench line only).  Profiles go to gpurun_out/ (tools/profile_model.sh) and are
# copied into this box's profiles/ so the bench line that follows reads its own PMC summary.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp ROUND=${ROUND:-r03}
mkdir -p gpurun_out
for c in "$@"; do
  only_bench=0
  if [ "${c%%:*}" = "bench" ]; then only_bench=1; c=${c#bench:}; fi
  M=${c%%:*}; S=""
  [ "$M" != "$c" ] && S=${c#*:}
  tag=$M; sarg=""
  if [ -n "$S" ]; then tag=${M}_$(echo "$S" | tr 'A-Z' 'a-z'); sarg="--solver $S"; fi
  if [ $only_bench -eq 0 ]; then
    bash tools/profile_model.sh $M $S || exit $?
    cp gpurun_out/pmc_${tag}_${ROUND}.json profiles/ || exit $?
  fi
  cpu=1
  [ "$M" = "cloth" ] && cpu=0
  timeout -k 10 400 python3 -u bench.py --model $M $sarg --cpu-baseline $cpu > gpurun_out/${ROUND}_bench_${tag}.log 2>&1 || exit $?
  python3 - "$tag" "gpurun_out/${ROUND}_bench_${tag}.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]).read().splitlines() if l.startswith("{")][-1])
r = d["roofline"]
print(sys.argv[1], round(d["value"], 1), "ms/step", round(d["ms_per_step"], 4), "group", r["group"], "kernel_ms", round(r["kernel_ms"], 4),
      "frac", round(r["frac"], 4), "traffic", r["traffic"], "src", r.get("traffic_source"), "cpu", (d.get("cpu_baseline") or {}).get("value"), flush=True)
PY
done
exit 0
