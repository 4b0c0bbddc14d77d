#!/bin/bash
# forward-kernel occupancy sensitivity: MJW_LDS_PAD adds LDS per world to the forward kernel, lowering
# the worlds (waves) per CU from the 16 the VGPR cap allows; one bench line per pad
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for pad in 0 1100 2000 3800 5000 8300 10700; do
  MJW_LDS_PAD=$pad timeout -k 10 200 python bench.py --steps 500 --cpu-baseline 0 > gpurun_out/occ_$pad.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/occ_$pad.log').read().strip().splitlines()[-1]); print(json.dumps({'lds_pad_bytes': $pad, 'lds_per_world': 9840 + $pad, 'worlds_per_cu': min(16, 163840 // (9840 + $pad)), 'env_steps_per_s': d['value'], 'forward_kernel_ms': d['roofline']['kernel_ms']}))"
done
