#!/bin/bash
# round-5 A/B: fused whole-step kernel vs split on humanoid Newton (driver window and 200 steps)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for r in 1 2; do
EXTRA="--solver NEWTON" MODEL=humanoid timeout -k 10 600 bash tools/ab_libenv.sh 20 "-|" "-|MJW_FUSED=0" || exit 1
done
EXTRA="--solver NEWTON" MODEL=humanoid timeout -k 10 600 bash tools/ab_libenv.sh 200 "-|" "-|MJW_FUSED=0" || exit 1
