#!/bin/bash
# Round-4 closing GPU run: the whole -m gpu suite, then -- only when pytest ended normally (rc 0 / 1) --
# the profiles and bench lines of every config (tools/r04_measure.sh) and the driver-style 20-step line.
cd "$(dirname "$0")/.." || exit 1
NOBENCH=1 bash tools/r04_check.sh
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/r04_measure.sh "humanoid aloha_cloth" "humanoid humanoid:NEWTON franka apollo cloth aloha_cloth" || exit $?
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/bench20.log 2>&1 || exit $?
tail -1 gpurun_out/bench20.log | cut -c1-300
exit $rc
