#!/bin/bash
# Round 5: PMC + SQ + kernel-stats profiles of the other configs on the final sources (tools/profile_model.sh)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for spec in "franka" "apollo" "cloth" "aloha_cloth" "humanoid NEWTON"; do
  ROUND=r05 timeout -k 10 600 bash tools/profile_model.sh $spec > gpurun_out/prof_$(echo $spec | tr ' ' '_').log 2>&1 || { tail -5 gpurun_out/prof_$(echo $spec | tr ' ' '_').log; exit 1; }
  tail -1 gpurun_out/prof_$(echo $spec | tr ' ' '_').log
done
