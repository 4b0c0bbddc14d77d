"""Muscle actuators (forward.py:671-727, util_misc.py:454-600): the <muscle> element, its length range,
the oracle against the curves' defining values, and the HIP path against the oracle."""

import numpy as np
import pytest

from tests.common import gpu_from_state, np_, oracle_from_state

XML = """<mujoco><compiler angle="radian"/><option timestep="0.005" gravity="0 0 -9.81"/>
<worldbody>
  <body pos="0 0 1"><joint name="j0" type="hinge" axis="0 1 0" range="-1 1.2" limited="true" damping="0.1"/>
    <geom type="capsule" fromto="0 0 0 0 0 -0.4" size="0.04" contype="0" conaffinity="0"/>
    <body pos="0 0 -0.4"><joint name="j1" type="hinge" axis="0 1 0" range="-1.5 0.5" limited="true"/>
      <geom type="capsule" fromto="0 0 0 0 0 -0.4" size="0.04" contype="0" conaffinity="0"/>
    </body>
  </body>
</worldbody>
<actuator>
  <muscle name="m0" joint="j0" ctrlrange="0 1" ctrllimited="true"/>
  <muscle name="m1" joint="j1" gear="2" ctrlrange="0 1" ctrllimited="true" force="30" timeconst="0.02 0.06" tausmooth="0.2"/>
  <motor joint="j1" gear="5"/>
</actuator></mujoco>"""


def _model():
  from mujoco_warp_amd import mjcf

  return mjcf.load_model_from_string(XML)


def test_compiler_muscle_fields():
  mjm = _model()
  assert list(mjm.actuator_gaintype[:2]) == [2, 2] and list(mjm.actuator_biastype[:2]) == [2, 2]
  assert list(mjm.actuator_dyntype) == [4, 4, 0] and mjm.na == 2
  np.testing.assert_allclose(mjm.actuator_gainprm[0, :9], [0.75, 1.05, -1, 200, 0.5, 1.6, 1.5, 1.3, 1.2])
  np.testing.assert_allclose(mjm.actuator_dynprm[1, :3], [0.02, 0.06, 0.2])
  np.testing.assert_allclose(mjm.actuator_gainprm[1, 2], 30.0)
  # length range = joint range x gear (gear 2 on j1)
  np.testing.assert_allclose(mjm.actuator_lengthrange[0], [-1.0, 1.2])
  np.testing.assert_allclose(mjm.actuator_lengthrange[1], [-3.0, 1.0])
  assert mjm.actuator_acc0[0] > 0


def test_oracle_muscle_force_at_optimal_length():
  """At the length whose normalized value is 1 and zero velocity the active curve is 1 (FL(1) = FV(0) =
  1) and the passive force 0, so force = -F act with F = scale / acc0 for force < 0 (util_misc.py:478-515);
  the activation rate from act = 0 at full excitation is 1 / (tau_act * 0.5)."""
  mjm = _model()
  from oracle import orc

  lr = mjm.actuator_lengthrange[0]
  L0 = (lr[1] - lr[0]) / (1.05 - 0.75)
  q = lr[0] + (1.0 - 0.75) * L0  # actuator length = q for gear 1
  od = orc.OracleData(orc.OracleModel(mjm), 1, 8, 8)
  od.qpos[0, 0] = q
  od.act[0] = [0.4, 0.0]
  od.ctrl[0] = [1.0, 0.0, 0.0]
  od.forward()
  F = 200.0 / mjm.actuator_acc0[0]
  np.testing.assert_allclose(od.actuator_force[0, 0], -F * 0.4, rtol=1e-12)
  np.testing.assert_allclose(od.act_dot[0, 0], (1.0 - 0.4) / (0.01 * (0.5 + 1.5 * 0.4)), rtol=1e-12)
  # stretched beyond optimum the passive force appears (negative, pulling back)
  od.qpos[0, 0] = lr[1]
  od.act[0] = [0.0, 0.0]
  od.forward()
  assert od.actuator_force[0, 0] < 0


@pytest.mark.gpu
def test_gpu_muscles_match_oracle():
  import torch

  import mujoco_warp_amd as mjw
  from tests.test_gpu_parity_strict import normwise_close

  mjm = _model()
  nworld = 8
  rng = np.random.default_rng(6)
  qpos = rng.uniform(-0.8, 0.4, (nworld, mjm.nq))
  qvel = rng.normal(0, 1.0, (nworld, mjm.nv))
  ctrl = rng.uniform(0, 1, (nworld, mjm.nu))
  act = rng.uniform(0, 1, (nworld, mjm.na))
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=16, nconmax=4)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=16, nconmax=4)
  d.act[:] = torch.as_tensor(act, dtype=torch.float32, device="cuda")
  od.act[:] = act
  mjw.fwd_position(m, d)
  mjw.fwd_velocity(m, d)
  mjw.fwd_actuation(m, d)
  od.fwd_position()
  od.fwd_velocity()
  od.fwd_actuation()
  torch.cuda.synchronize()
  from tests.test_gpu_parity_strict import strict_close

  strict_close("actuator_force", np_(d.actuator_force), od.actuator_force)
  strict_close("act_dot", np_(d.act_dot), od.act_dot)
  for _ in range(5):
    mjw.step(m, d)
    od.step()
  torch.cuda.synchronize()
  normwise_close("qpos", np_(d.qpos), od.qpos)
  normwise_close("act", np_(d.act), od.act)
  normwise_close("qvel", np_(d.qvel), od.qvel, tol=5e-3)
