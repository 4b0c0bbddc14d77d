#!/bin/bash
# Round 5 end-of-round measurement, part A (humanoid, the headline config): rocprof stats + PMC passes
# (tools/profile_model.sh -> pmc_humanoid_r05.json, bound to the sources' hash and copied into profiles/
# so that the bench line prices its traffic), the driver-style window (tools/r05_window.sh: bench line
# + rocprof kernel trace of the same command) and the default bench line with its CPU baseline.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
ROUND=r05 timeout -k 10 700 bash tools/profile_model.sh humanoid > gpurun_out/prof_humanoid.log 2>&1 || { tail -5 gpurun_out/prof_humanoid.log; exit 1; }
cp gpurun_out/pmc_humanoid_r05.json profiles/ || exit 1
timeout -k 10 500 bash tools/r05_window.sh humanoid 20 5 > gpurun_out/window_humanoid.txt 2>&1 || { tail -5 gpurun_out/window_humanoid.txt; exit 1; }
cat gpurun_out/window_humanoid.txt
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_humanoid.log 2>&1 || { tail -5 gpurun_out/bench_humanoid.log; exit 1; }
tail -1 gpurun_out/bench_humanoid.log | cut -c1-600
