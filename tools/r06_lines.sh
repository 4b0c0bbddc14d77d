#!/bin/bash
# Round 6: one bench line per config on the final sources (two runs each), for BASELINE.md.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for args in "--steps 20 --warmup 5" "--steps 1000 --warmup 20" "--steps 1000 --warmup 20 --solver NEWTON" "--model franka" "--model apollo" "--model aloha_cloth" "--model cloth"; do
  for rep in 1 2; do
    timeout -k 10 300 python -u bench.py $args --cpu-baseline 0 < /dev/null > gpurun_out/lines.log 2>&1 || { tail -3 gpurun_out/lines.log; exit 1; }
    tail -1 gpurun_out/lines.log >> gpurun_out/r06_lines.jsonl
    echo "[$args] rep $rep: $(python3 -c "import json,sys;d=json.loads(open('gpurun_out/lines.log').read().splitlines()[-1]);r=d['roofline'];print(round(d['value']/1e6,4),'M', round(d['ms_per_step'],4), r['group'], round(r['kernel_ms'],4), round(r['frac'],4), r['groups'][r['group']].get('traffic_over_alg'))")"
  done
done
exit 0
