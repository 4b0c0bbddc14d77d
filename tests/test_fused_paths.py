"""The fused whole-step kernel (step_kernel: the forward stages and the dense CG solve of a world in one wave,
the default for lean humanoid-class CG models) against the two-kernel path it replaces (MJW_FUSED=0: forward
kernel, then dense kernel), which still serves Newton, box, sensor and CCD models.

MJW_FUSED is read once per process (a static in the launcher), so each path runs in a subprocess of its own;
both step the same seeded humanoid states and write their outputs to an .npz for comparison.  The two
paths compute the same stages in the same order, so they agree to fp32 rounding: qpos normwise 1e-5 and
qvel / efc_force at the solver bar after a few steps (tests/test_gpu_parity_models.py's bars).
"""

import os
import subprocess
import sys

import numpy as np
import pytest

from tests.common import ROOT

CHILD = r"""
import sys, numpy as np, torch
sys.path.insert(0, {root!r})
import mujoco_warp_amd as mjw
from tests.common import humanoid_model, random_states, gpu_from_state, np_
mjm = humanoid_model("CG")
qpos, qvel, ctrl = random_states(mjm, 64, seed=11)
m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=64, nconmax=24)
for _ in range({nstep}):
  mjw.step(m, d)
torch.cuda.synchronize()
np.savez({out!r}, qpos=np_(d.qpos), qvel=np_(d.qvel), efc_force=np_(d.efc.force), nefc=d.nefc.cpu().numpy(),
         niter=d.solver_niter.cpu().numpy())
"""


def _run(tmp_path, fused, nstep):
  out = str(tmp_path / f"fused{fused}.npz")
  env = dict(os.environ)
  env["MJW_FUSED"] = "1" if fused else "0"
  code = CHILD.format(root=ROOT, nstep=nstep, out=out)
  subprocess.run([sys.executable, "-c", code], check=True, env=env, cwd=ROOT, timeout=300)
  return np.load(out)


@pytest.mark.gpu
def test_gpu_fused_step_matches_two_kernel_path(tmp_path):
  a = _run(tmp_path, True, 3)
  b = _run(tmp_path, False, 3)
  np.testing.assert_array_equal(a["nefc"], b["nefc"])
  e = np.linalg.norm(a["qpos"] - b["qpos"], axis=1) / np.linalg.norm(b["qpos"], axis=1)
  assert e.max() < 1e-5, e.max()
  ev = np.linalg.norm(a["qvel"] - b["qvel"], axis=1) / (np.linalg.norm(b["qvel"], axis=1) + 1.0)
  assert ev.max() < 5e-3, ev.max()
  for w in range(a["qpos"].shape[0]):
    n = int(a["nefc"][w])
    fa, fb = a["efc_force"][w, :n], b["efc_force"][w, :n]
    assert np.linalg.norm(fa - fb) <= 5e-3 * (np.linalg.norm(fb) + 1.0), w
  print(f"fused vs two-kernel: qpos {e.max():.2e}, qvel {ev.max():.2e}, bitwise equal worlds "
        f"{int((a['qpos'] == b['qpos']).all(axis=1).sum())} / {a['qpos'].shape[0]}")
