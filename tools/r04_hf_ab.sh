#!/bin/bash
# GPU check of one round-4 change: the selected tests (PYTEST_K), then -- only when pytest itself ended
# normally (rc 0 / 1: no fault, abort or timeout) -- the A/B bench against the variant library.
cd "$(dirname "$0")/.." || exit 1
NOBENCH=1 bash tools/r04_check.sh
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/ab_libenv.sh "${AB_STEPS:-300}" "mujoco_warp_amd/libmjw_amd_old.so|" "-|" "mujoco_warp_amd/libmjw_amd_old.so|" "-|" || exit $?
exit $rc
