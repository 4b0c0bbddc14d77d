#!/bin/bash
# A/B of library variants on the headline bench: bash tools/ab_bench.sh [steps] lib1.so lib2.so ...
# (the default build first); one JSON line per variant into gpurun_out/ab_<name>.log
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
STEPS=$1; shift
MODEL=${MODEL:-humanoid}
timeout -k 10 200 python -u bench.py --model $MODEL --steps $STEPS --cpu-baseline 0 > gpurun_out/ab_default.log 2>&1 || exit $?
echo "default: $(python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab_default.log').read().splitlines()[-1]);print(round(d['value']/1e6,3),'M', round(d['roofline']['kernel_ms'],4), round(d['roofline']['other_kernels'][list(d['roofline']['other_kernels'])[0]]['ms'],4))")"
for lib in "$@"; do
  n=$(basename $lib .so)
  MJW_LIB_PATH=$PWD/$lib timeout -k 10 200 python -u bench.py --model $MODEL --steps $STEPS --cpu-baseline 0 > gpurun_out/ab_$n.log 2>&1 || exit $?
  echo "$n: $(python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab_$n.log').read().splitlines()[-1]);print(round(d['value']/1e6,3),'M', round(d['roofline']['kernel_ms'],4), round(d['roofline']['other_kernels'][list(d['roofline']['other_kernels'])[0]]['ms'],4))")"
done
