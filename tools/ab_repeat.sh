#!/bin/bash
# interleaved repeats of bench variants within one GPU call: bash tools/ab_repeat.sh NREP "args1" "args2" ...
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
N=$1; shift
for r in $(seq 1 $N); do
  i=0
  for a in "$@"; do
    timeout -k 10 200 python -u bench.py --cpu-baseline 0 $a > gpurun_out/abr_$i.log 2>&1 || exit $?
    echo "rep $r [$a]: $(python3 -c "import json;d=json.loads(open('gpurun_out/abr_$i.log').read().splitlines()[-1]);r=d['roofline'];print(round(d['value']/1e6,3),'M', round(d['ms_per_step'],4), 'fwd', round(r['kernel_ms'],4), 'frac', round(r['frac'],4))")"
    i=$((i+1))
  done
done
