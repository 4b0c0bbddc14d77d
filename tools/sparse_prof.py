"""Per-phase in-kernel timing of the sparse / flex path (mjw_sparse.hip, s_memtime deltas summed over
waves) on the cloth or aloha_cloth benchmark.

Builds mujoco_warp_amd/libmjw_amd_prof.so with -DMJW_PROFILE (unless present) and loads it via
MJW_LIB_PATH.  usage: python tools/sparse_prof.py [cloth|aloha_cloth] [nworld] [nsteps] [warmup]
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PROF = os.path.join(ROOT, "mujoco_warp_amd", "libmjw_amd_prof.so")
if not os.path.exists(PROF):
  from mujoco_warp_amd import build

  build.build(out=PROF, defines=("MJW_PROFILE",))
os.environ["MJW_LIB_PATH"] = PROF

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import mujoco_warp_amd as mjw  # noqa: E402
from mujoco_warp_amd import _lib, mjcf  # noqa: E402

PHASES = ["kinematics+com+camlight", "flex_edges", "crb_qM", "collision", "make_constraint+transmission", "fwd_velocity",
          "fwd_actuation", "fwd_acceleration", "solve_init", "solve_linesearch", "solve_update", "solve_cg_tail"]
which = sys.argv[1] if len(sys.argv) > 1 else "aloha_cloth"
cfg = bench.MODELS[which]
nworld = int(sys.argv[2]) if len(sys.argv) > 2 else cfg["nworld"]
nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
warmup = int(sys.argv[4]) if len(sys.argv) > 4 else 20
mjm = mjcf.load_model(os.path.join(ROOT, cfg["path"]))
mjd = mjcf.MjData(mjm)
center = None
if cfg["key"] is not None:
  mjcf.reset_data_keyframe(mjm, mjd, cfg["key"])
  center = torch.as_tensor(np.asarray(mjm.key_ctrl[cfg["key"]], dtype=np.float32), device="cuda")
m = mjw.put_model(mjm, device="cuda")
d = mjw.put_data(mjm, mjd, nworld=nworld, nconmax=cfg["nconmax"], njmax=cfg["njmax"], device="cuda", m=m)
L = _lib.lib()
SUB = ["cg:mul_m", "cg:jv_pass", "cg:ls_passes", "cg:constraint_rows", "cg:JTf", "cg:precondition"]
buf = (ctypes.c_ulonglong * (len(PHASES) + 2 + len(SUB)))()  # + the line-search row-pass and CG-iteration counts, sub-phases
for i in range(warmup):
  mjw.ctrl_noise(m, d, i, center=center)
  mjw.step(m, d)
torch.cuda.synchronize()
L.mjw_prof_read_sparse(buf, 1)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for i in range(nsteps):
  mjw.ctrl_noise(m, d, warmup + i, center=center)
  mjw.step(m, d)
e1.record()
torch.cuda.synchronize()
L.mjw_prof_read_sparse(buf, 0)
npass, niter = buf[len(PHASES)], buf[len(PHASES) + 1]
tot = sum(buf[:len(PHASES)]) or 1
out = {"model": which, "nworld": nworld, "ms_per_step": e0.elapsed_time(e1) / nsteps,
       "nefc_mean": float(d.nefc.float().mean()), "solver_niter_mean": float(d.solver_niter.float().mean()),
       "cg_iterations_per_world_step": niter / (nworld * nsteps),
       "linesearch_row_passes_per_cg_iteration": npass / max(niter, 1),
       "wave_cycles_per_world_step": {p: buf[i] / (nworld * nsteps) for i, p in enumerate(PHASES)},
       "share": {p: round(buf[i] / tot, 4) for i, p in enumerate(PHASES)},
       "cg_subphase_cycles_per_world_step": {p: buf[len(PHASES) + 2 + i] / (nworld * nsteps) for i, p in enumerate(SUB)},
       "cg_subphase_share_of_total": {p: round(buf[len(PHASES) + 2 + i] / tot, 4) for i, p in enumerate(SUB)}}
print(json.dumps(out, indent=1))
