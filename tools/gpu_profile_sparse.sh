#!/bin/bash
# rocprofv3 passes for a sparse-path model (default aloha_cloth): kernel-trace stats of a short bench,
# then FETCH_SIZE and WRITE_SIZE in separate passes (never combined with trace domains).
cd "$(dirname "$0")/.." || exit 1
M=${1:-aloha_cloth}
R=${ROUND:-r02}
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/sprof_stats gpurun_out/sprof_fetch gpurun_out/sprof_write
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sprof_stats -o run -- python3 bench.py --model $M --steps 20 --warmup 10 --cpu-baseline 0 --graph 0 > gpurun_out/sprof_stats.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/sprof_fetch -o run -- python3 bench.py --model $M --steps 5 --warmup 10 --cpu-baseline 0 --graph 0 > gpurun_out/sprof_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/sprof_write -o run -- python3 bench.py --model $M --steps 5 --warmup 10 --cpu-baseline 0 --graph 0 > gpurun_out/sprof_write.log 2>&1 || exit $?
python3 tools/pmc_traffic.py gpurun_out/sprof_stats gpurun_out/sprof_fetch gpurun_out/sprof_write gpurun_out/pmc_${M}_$R.json ${NWL:-1024} CG $M || exit $?
find gpurun_out/sprof_stats -name "*kernel_stats.csv" -exec cp {} gpurun_out/${R}_${M}_kernel_stats.csv \;
exit 0
