"""Per-phase in-kernel timing (s_memtime deltas summed over waves) of the humanoid step.

Builds mujoco_warp_amd/libmjw_amd_prof.so with -DMJW_PROFILE (unless present), loads it via
MJW_LIB_PATH, runs `nsteps` steps of the benchmark workload and prints each phase's share.
usage: python tools/phase_prof.py [nworld] [nsteps] [CG|NEWTON|default] [model]
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

import torch  # noqa: E402

import mujoco_warp_amd as mjw  # noqa: E402
from mujoco_warp_amd import _lib, mjcf  # noqa: E402

PHASES = ["load", "kinematics", "com_pos", "camlight", "crb_qM", "collision+constraints", "transmission", "fwd_velocity",
          "fwd_actuation", "fwd_acceleration", "generic_solve", "generic_euler", "dense_factor", "dense_solve", "dense_euler"]
# sub-phases of collision+constraints (not part of the total)
SUB = ["c:eq_friction_limits", "c:broadphase", "c:narrowphase_staging", "c:pool_write", "c:contact_J", "c:row_scalars", "c:tail",
       "newton:H_build", "newton:H_cholesky"]
nworld = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 100
solver = sys.argv[3] if len(sys.argv) > 3 else "CG"
model = sys.argv[4] if len(sys.argv) > 4 else "humanoid"  # a bench.py config (dense-path models)
warm = int(sys.argv[5]) if len(sys.argv) > 5 else 20  # 5: the driver's bench window (steps 5..5+nsteps)
from bench import MODELS  # noqa: E402

cfg = MODELS[model]
mjm = mjcf.load_model(os.path.join(ROOT, cfg["path"]))
if solver != "default":
  mjw.override_model(mjm, [f"opt.solver={solver}"])
mjd = mjcf.MjData(mjm)
if cfg["key"] is not None:
  mjcf.reset_data_keyframe(mjm, mjd, cfg["key"])
m = mjw.put_model(mjm, device="cuda")
d = mjw.put_data(mjm, mjd, nworld=nworld, nconmax=cfg["nconmax"], njmax=cfg["njmax"], device="cuda", m=m)
center = None if cfg["key"] is None else torch.as_tensor(mjm.key_ctrl[cfg["key"]], dtype=torch.float32, device="cuda")
L = _lib.lib()
buf = (ctypes.c_ulonglong * (len(PHASES) + len(SUB)))()
for i in range(warm):
  mjw.ctrl_noise(m, d, i, center=center)
  mjw.step(m, d)
torch.cuda.synchronize()
L.mjw_prof_read(buf, 1)
L.mjw_prof_read_dense(buf, 1)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for i in range(nsteps):
  mjw.ctrl_noise(m, d, warm + i, center=center)
  mjw.step(m, d)
e1.record()
torch.cuda.synchronize()
a = (ctypes.c_ulonglong * (len(PHASES) + len(SUB)))()
b = (ctypes.c_ulonglong * (len(PHASES) + len(SUB)))()
L.mjw_prof_read(a, 0)
L.mjw_prof_read_dense(b, 0)
tot = [a[i] + b[i] for i in range(len(PHASES))]
s = sum(tot) or 1
out = {"nworld": nworld, "solver": solver, "ms_per_step": e0.elapsed_time(e1) / nsteps,
       "wave_cycles_per_world_step": {p: tot[i] / (nworld * nsteps) for i, p in enumerate(PHASES) if tot[i]},
       "share": {p: round(tot[i] / s, 4) for i, p in enumerate(PHASES) if tot[i]},
       "subphase_cycles_per_world_step": {p: (a[len(PHASES) + i] + b[len(PHASES) + i]) / (nworld * nsteps) for i, p in enumerate(SUB)}}
print(json.dumps(out, indent=1))
