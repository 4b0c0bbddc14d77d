#!/bin/bash
# rocprofv3 passes of one bench config for profiles/: kernel-trace stats, then FETCH_SIZE, WRITE_SIZE
# and the SQ counters in separate passes (never combined with trace domains), then the per-kernel /
# per-step traffic summary (tools/pmc_traffic.py) tagged with the kernel sources' hash.
# usage: ROUND=r03 bash tools/profile_model.sh <model> [solver]   -> gpurun_out/pmc_<model>[_<solver>]_<round>.json
cd "$(dirname "$0")/.." || exit 1
M=${1:-humanoid}
S=${2:-}
R=${ROUND:-r05}
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=$M
sarg=""
if [ -n "$S" ]; then tag=${M}_$(echo "$S" | tr 'A-Z' 'a-z'); sarg="--solver $S"; fi
read -r NW SOLVER < <(python3 -c "
import bench, sys
sys.argv = ['bench.py', '--model', '$M'] + ('$sarg'.split())
a = bench.parse()
import mujoco_warp_amd as mjw
s = a.solver or {1: 'CG', 2: 'NEWTON'}[int(mjw.load_model(bench.MODELS['$M']['path']).opt.solver)]
print(a.nworld, s)") || exit 1
# The counter passes (FETCH_SIZE, WRITE_SIZE, SQ) run the driver's own command -- `bench.py --steps 20
# --warmup 5`, the timed region replayed as a hipGraph -- followed by bench.py's trace pass, which replays
# that window eagerly from the state saved at its start: the summary averages exactly the trace pass (tail =
# its steps), whose nefc / ncon the pass's bench line reports, so bench.py prices the driver window's
# algorithmic bytes (round 6; round 5 counted a later, contact-richer window after 200 eager warm-up steps).
# The stats pass runs the same window (the kernel-time averages of the line's `achieved`).  The flex configs
# count 5 steps after 20 (their steps take ~20 ms).
steps_stats=20; warm_stats=5; steps_pmc=20; warm_pmc=5
case $M in aloha_cloth|cloth) steps_stats=20; warm_stats=20; steps_pmc=5; warm_pmc=20;; esac
common="--model $M $sarg --cpu-baseline 0"
d=gpurun_out/prof_$tag
rm -rf $d && mkdir -p $d
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $d/stats -o run -- python3 bench.py $common --steps $steps_stats --trace-steps $steps_stats --warmup $warm_stats > $d/stats.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $d/fetch -o run -- python3 bench.py $common --steps $steps_pmc --trace-steps $steps_pmc --warmup $warm_pmc > $d/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $d/write -o run -- python3 bench.py $common --steps $steps_pmc --trace-steps $steps_pmc --warmup $warm_pmc > $d/write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d $d/sq -o run -- python3 bench.py $common --steps $steps_pmc --trace-steps $steps_pmc --warmup $warm_pmc > $d/sq.log 2>&1 || exit $?
python3 tools/sq_counters.py $d/sq > gpurun_out/${R}_${tag}_sq_counters.txt || exit $?
python3 tools/pmc_traffic.py $d/stats $d/fetch $d/write gpurun_out/pmc_${tag}_$R.json $NW $SOLVER $M $steps_pmc > $d/pmc.log || exit $?
find $d/stats -name "*kernel_stats.csv" -exec cp {} gpurun_out/${R}_${tag}_kernel_stats.csv \;
echo "profiled $tag nworld=$NW solver=$SOLVER"
exit 0
