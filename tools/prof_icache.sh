#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
grep -E "ICACHE|IFETCH|SQ_INST_|SQ_INSTS_|LDS_BANK|SQ_BUSY|SQ_WAIT" gpurun_out/counters_list.txt | head -80 > gpurun_out/counters_sel.txt
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_IFETCH --output-format csv -d gpurun_out/pmc_sq1 -o run -- python3 bench.py --steps 20 --warmup 10 --cpu-baseline 0 > gpurun_out/pmc_sq1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM --output-format csv -d gpurun_out/pmc_sq2 -o run -- python3 bench.py --steps 20 --warmup 10 --cpu-baseline 0 > gpurun_out/pmc_sq2.log 2>&1 || exit $?
python3 tools/sq_counters.py gpurun_out/pmc_sq1 > gpurun_out/sq1.txt 2>&1
python3 tools/sq_counters.py gpurun_out/pmc_sq2 > gpurun_out/sq2.txt 2>&1
cat gpurun_out/sq1.txt gpurun_out/sq2.txt
