"""deriv_smooth_vel (derivative.py:321-416) and set_length_range (io.py:2465-2495, _set_length_range
:2158-2194), the reference entry points around the implicitfast integrator and the muscle length ranges.

CPU: set_length_range against the reference kernel's rule (limited joint / tendon range times gear[0],
swapped for a negative gear, (0, 0) otherwise), per world.  `-m gpu`: after a device forward,
deriv_smooth_vel's qM - dt qDeriv against the fp64 oracle's qM and a central finite difference of the
oracle's qfrc_actuator + qfrc_passive in qvel, on slide-joint chains (no velocity-dependent bias, whose
derivative the reference leaves out too) with affine position / velocity actuators, dof and tendon damping,
on the dense and the sparse path."""

import numpy as np
import pytest

from tests.common import gpu_from_state, np_, oracle_from_state

RANGE_XML = """<mujoco><worldbody>
<body><joint name="j0" type="slide" axis="1 0 0" limited="true" range="-.2 .3"/><geom size=".1"/>
  <body pos="0 0 -.3"><joint name="j1" type="hinge" axis="0 1 0" limited="true" range="-30 60"/><geom size=".1"/>
    <body pos="0 0 -.3"><joint name="j2" type="hinge" axis="1 0 0"/><geom size=".1"/><site name="s"/></body></body></body>
</worldbody>
<tendon><fixed name="t" limited="true" range="-.1 .4"><joint joint="j0" coef="1"/><joint joint="j1" coef="-.5"/></fixed></tendon>
<actuator><position joint="j0" kp="10" gear="2"/><motor joint="j1" gear="-3"/><motor joint="j2"/>
  <motor tendon="t" gear="-1.5"/><motor site="s" gear="1 0 0 0 0 0"/></actuator></mujoco>"""


def test_set_length_range_rule():
  import torch

  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf

  mjm = mjcf.load_model_from_string(RANGE_XML)
  m = mjw.put_model(mjm, device="cpu")
  d = mjw.make_data(mjm, nworld=2, nconmax=4, njmax=8, device="cpu", m=m)
  mjw.set_length_range(m, d)
  lr = m.actuator_lengthrange.reshape(-1, mjm.nu, 2).double().numpy()
  d2r = np.pi / 180
  want = np.array([[-0.4, 0.6], [-60 * d2r * 3, 30 * d2r * 3], [0, 0], [-0.6, 0.15], [0, 0]])
  for w in range(lr.shape[0]):
    np.testing.assert_allclose(lr[w], want, rtol=1e-6, atol=1e-7)
  # per-world gear: world 1 doubles actuator 0's gear
  gear = torch.as_tensor(np.stack([mjm.actuator_gear, mjm.actuator_gear]), dtype=torch.float32)
  gear[1, 0, 0] = 4.0
  m.actuator_gear = gear
  mjw.set_length_range(m, d)
  lr = m.actuator_lengthrange.reshape(-1, mjm.nu, 2).double().numpy()
  np.testing.assert_allclose(lr[1, 0], [-0.8, 1.2], rtol=1e-6)
  np.testing.assert_allclose(lr[0, 0], [-0.4, 0.6], rtol=1e-6)


SLIDES = """<mujoco><option timestep="0.01" jacobian="{jac}" integrator="implicitfast"/><worldbody>
<body><joint name="a" type="slide" axis="1 0 0" damping=".3"/><geom size=".1" contype="0" conaffinity="0"/>
  <body pos="0 0 -.3"><joint name="b" type="slide" axis="0 1 0" damping=".2"/><geom size=".1" contype="0" conaffinity="0"/>
    <body pos="0 0 -.3"><joint name="c" type="slide" axis="0 .6 .8" damping=".1"/><geom size=".1" contype="0" conaffinity="0"/></body></body></body>
<body pos="1 0 0"><joint name="d" type="slide" axis="0 0 1"/><geom size=".1" contype="0" conaffinity="0"/></body>
</worldbody>
<tendon><fixed name="t" damping=".7"><joint joint="a" coef="1"/><joint joint="c" coef="-.5"/></fixed></tendon>
<actuator><position joint="a" kp="40" kv="3"/><velocity joint="b" kv="2"/><general joint="c" gainprm="1 0 .5" biasprm="0 0 -.4" gaintype="affine" biastype="affine"/>
  <position tendon="t" kp="5" kv="1.5"/><intvelocity joint="d" kp="3" actrange="-1 1"/></actuator></mujoco>"""


@pytest.mark.gpu
@pytest.mark.parametrize("jac", ["dense", "sparse"])
def test_gpu_deriv_smooth_vel_matches_finite_difference(jac):
  import torch

  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf

  mjm = mjcf.load_model_from_string(SLIDES.format(jac=jac))
  nworld = 4
  rng = np.random.default_rng(9)
  qpos = rng.normal(0, 0.2, (nworld, mjm.nq))
  qvel = rng.normal(0, 1.0, (nworld, mjm.nv))
  ctrl = rng.uniform(-0.5, 0.5, (nworld, mjm.nu))
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=8, nconmax=4)
  assert m.is_sparse == (jac == "sparse")
  mjw.forward(m, d)
  out = torch.zeros_like(d.qM)
  mjw.deriv_smooth_vel(m, d, out)
  torch.cuda.synchronize()
  nv, dt, eps = mjm.nv, mjm.opt.timestep, 1e-6
  from tests.parity_models import dense_M

  def smooth(v):
    _, od = oracle_from_state(mjm, qpos, v, ctrl, njmax=8, nconmax=4)
    od.forward()
    return od, od.qfrc_actuator + od.qfrc_passive

  od, _ = smooth(qvel)
  for w in range(nworld):
    fd = np.zeros((nv, nv))
    for j in range(nv):
      vp, vm = qvel.copy(), qvel.copy()
      vp[w, j] += eps
      vm[w, j] -= eps
      fd[:, j] = (smooth(vp)[1][w] - smooth(vm)[1][w]) / (2 * eps)
    want = od.qM[w].reshape(nv, nv) - dt * fd
    if jac == "sparse":
      from tests.cloth_common import dense_qM

      got = dense_qM(mjm, np_(out[w]))
    else:
      got = np_(out[w])[:nv, :nv]
    # the reference fills the qM (ancestor) pattern only; d sits on its own tree
    want[3, :3] = want[:3, 3] = 0.0
    np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-5 * np.abs(want).max())
