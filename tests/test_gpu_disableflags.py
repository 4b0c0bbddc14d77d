"""Option.disableflags on the HIP path vs the fp64 oracle (the reference parameterises its forward /
smooth tests over these flags: forward_test.py:67-111, :128-135, :195-204).

Each flag is set on the humanoid (eulerdamp, which humanoid.xml disables, is re-enabled instead), one
step is taken from seeded random states with controls beyond ctrlrange and a nonzero warmstart, and the
constraint rows (count, order, type) and the stepped state are compared with the oracle.  The
tolerances are those of the round-1 rollout test (test_gpu_parity.py): the CG solution agrees to the
solver tolerance, not to fp32 rounding."""

import numpy as np
import pytest

from tests.common import assert_close, gpu_from_state, humanoid_model, np_, oracle_from_state, random_states

pytestmark = pytest.mark.gpu

FLAGS = {
  "constraint": 1 << 0,
  "frictionloss": 1 << 2,
  "limit": 1 << 3,
  "contact": 1 << 4,
  "spring": 1 << 5,
  "damper": 1 << 6,
  "gravity": 1 << 7,
  "clampctrl": 1 << 8,
  "warmstart": 1 << 9,
  "actuation": 1 << 11,
  "refsafe": 1 << 12,
  "eulerdamp_on": -(1 << 15),  # clear the bit humanoid.xml sets
}


@pytest.mark.parametrize("flag", sorted(FLAGS))
def test_disableflag_step_matches_oracle(flag):
  import torch

  import mujoco_warp_amd as mjw

  mjm = humanoid_model("CG")
  bit = FLAGS[flag]
  if bit > 0:
    mjm.opt.disableflags = int(mjm.opt.disableflags) | bit
  else:
    mjm.opt.disableflags = int(mjm.opt.disableflags) & ~(-bit)
  nworld = 8
  qpos, qvel, ctrl = random_states(mjm, nworld, seed=11, qvel_noise=0.3)
  ctrl = 2.0 * ctrl  # beyond ctrlrange [-1, 1]: clampctrl matters
  warm = np.random.default_rng(12).normal(0, 1.0, (nworld, mjm.nv))
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, qacc_warmstart=warm)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl, qacc_warmstart=warm)
  mjw.fwd_position(m, d)
  torch.cuda.synchronize()
  od.fwd_position()
  nefc = np_(d.nefc).astype(int)
  np.testing.assert_array_equal(nefc, od.nefc.reshape(-1).astype(int))
  for w in range(nworld):
    np.testing.assert_array_equal(d.efc.type[w, : nefc[w]].cpu().numpy(), od.efc_type[w, : nefc[w]])
  if flag in ("constraint", "contact"):
    assert int(d.nacon[0]) == 0 or flag == "constraint"
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, qacc_warmstart=warm)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl, qacc_warmstart=warm)
  mjw.step(m, d)
  torch.cuda.synchronize()
  od.step()
  assert np.isfinite(np_(d.qpos)).all()
  assert_close("qpos", np_(d.qpos), od.qpos, rtol=2e-3, atol=2e-3)
  scale = np.abs(od.qvel).max() + 1.0
  assert_close("qvel", np_(d.qvel), od.qvel, rtol=2e-2, atol=2e-2 * scale)
  assert_close("qfrc_smooth", np_(d.qfrc_smooth), od.qfrc_smooth, rtol=1e-3, atol=1e-3 * (np.abs(od.qfrc_smooth).max() + 1.0))
