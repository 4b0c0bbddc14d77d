#!/bin/bash
# Instruction-cache counters of the headline's fused step kernel (driver window), one small pass each.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cloth.py tests/test_gpu_parity_models.py tests/test_collision_stages.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_ic_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r06_ic_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --output-format csv -d gpurun_out/pmc_ic1 -o run -- python3 bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/pmc_ic1.log 2>&1 || { tail -3 gpurun_out/pmc_ic1.log; exit 1; }
python3 tools/sq_counters.py gpurun_out/pmc_ic1 > gpurun_out/ic1.txt 2>&1; cat gpurun_out/ic1.txt | head -30
timeout -s KILL 120 rocprofv3 --pmc SQ_IFETCH SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAVES --output-format csv -d gpurun_out/pmc_ic2 -o run -- python3 bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/pmc_ic2.log 2>&1 || { tail -3 gpurun_out/pmc_ic2.log; exit 1; }
python3 tools/sq_counters.py gpurun_out/pmc_ic2 > gpurun_out/ic2.txt 2>&1; cat gpurun_out/ic2.txt | head -30
exit 0
