#!/bin/bash
# rocprofv3 passes for the round's profiles/: kernel-trace stats of the bench command, then
# FETCH_SIZE and WRITE_SIZE in separate passes (never combined with trace domains).
cd "$(dirname "$0")/.." || exit 1
R=${ROUND:-r02}
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_stats gpurun_out/prof_fetch gpurun_out/prof_write gpurun_out/prof_sq
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stats -o run -- python3 bench.py --steps 200 --cpu-baseline 0 --graph 0 > gpurun_out/prof_stats.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch -o run -- python3 bench.py --steps 20 --warmup 10 --cpu-baseline 0 --graph 0 > gpurun_out/prof_fetch.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write -o run -- python3 bench.py --steps 20 --warmup 10 --cpu-baseline 0 --graph 0 > gpurun_out/prof_write.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d gpurun_out/prof_sq -o run -- python3 bench.py --steps 20 --warmup 10 --cpu-baseline 0 --graph 0 > gpurun_out/prof_sq.log 2>&1 || exit $?
python3 tools/sq_counters.py gpurun_out/prof_sq > gpurun_out/${R}_sq_counters.txt || exit $?
python3 tools/pmc_traffic.py gpurun_out/prof_stats gpurun_out/prof_fetch gpurun_out/prof_write gpurun_out/pmc_humanoid_$R.json ${NWL:-8192} || exit $?
find gpurun_out/prof_stats -name "*kernel_stats.csv" -exec cp {} gpurun_out/${R}_kernel_stats.csv \;
exit 0
