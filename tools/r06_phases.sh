#!/bin/bash
# Round 6: phase splits from the profile build (per-phase counters spread over 64 copies): humanoid CG and
# Newton on the driver window, aloha_cloth's sparse CG sub-phases.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/phase_prof.py 8192 20 CG humanoid 5 < /dev/null > gpurun_out/r06_phase_cg_final.log 2>&1 || { tail -5 gpurun_out/r06_phase_cg_final.log; exit 1; }
timeout -k 10 300 python -u tools/phase_prof.py 8192 20 NEWTON humanoid 5 < /dev/null > gpurun_out/r06_phase_newton_final.log 2>&1 || { tail -5 gpurun_out/r06_phase_newton_final.log; exit 1; }
timeout -k 10 300 python -u tools/sparse_prof.py aloha_cloth 1024 5 20 < /dev/null > gpurun_out/r06_sparse_prof_final.log 2>&1 || { tail -5 gpurun_out/r06_sparse_prof_final.log; exit 1; }
for f in r06_phase_cg_final r06_phase_newton_final r06_sparse_prof_final; do python3 -c "
import json,sys; t=open('gpurun_out/$f.log').read(); d=json.loads(t[t.index('{'):]); print('$f', d['ms_per_step'], d.get('share'), d.get('subphase_cycles_per_world_step') or d.get('cg_subphase_share_of_total'))"; done
exit 0
