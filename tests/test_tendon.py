"""Fixed (joint) tendons: length / Jacobian (smooth.py:3085-3121), velocity
(forward.py:604-609), armature in qM (smooth.py:916-1000), spring / damper (passive.py:183-252),
friction and limit rows (constraint.py:1204-1313, 1547-1665), tendon transmissions (smooth.py:2244-2260)
and the actuator force range of a tendon (forward.py:739-779).

The reference's tendon tests compare against MuJoCo C at run time, so the oracle restatement is pinned
by analytic cases here; `-m gpu` tests compare the HIP path with the oracle.
"""

import numpy as np
import pytest

from tests.common import gpu_from_state, np_, oracle_from_state

XML = """<mujoco><option gravity="0 0 {g}"/><worldbody>
<body><joint name="a" type="hinge" axis="0 1 0" {ja}/><geom type="capsule" size=".05" fromto="0 0 0 .3 0 0" mass="1"/>
  <body pos=".3 0 0"><joint name="b" type="hinge" axis="0 1 0"/><geom type="capsule" size=".05" fromto="0 0 0 .3 0 0" mass="1"/></body></body>
<body pos="0 1 0"><joint name="c" type="slide" axis="1 0 0"/><geom type="sphere" size=".1" mass="2"/></body>
</worldbody>
<tendon><fixed name="t" {ten}><joint joint="a" coef="1"/><joint joint="b" coef="-.5"/><joint joint="c" coef="2"/></fixed></tendon>
<actuator><motor tendon="t" gear="2" {act}/><motor joint="a"/></actuator></mujoco>"""


def _model(g=0.0, ja="", ten="", act=""):
  from mujoco_warp_amd import mjcf

  return mjcf.load_model_from_string(XML.format(g=g, ja=ja, ten=ten, act=act))


def _od(mjm, qpos, qvel, ctrl=None, njmax=16):
  n = qpos.shape[0]
  return oracle_from_state(mjm, qpos, qvel, np.zeros((n, mjm.nu)) if ctrl is None else ctrl, njmax=njmax, nconmax=4)[1]


def test_compiler_fields():
  m = _model(ten='stiffness="10" springlength="0.1 0.3" range="-1 1" frictionloss=".2" armature=".05"')
  assert m.ntendon == 1 and m.nwrap == 3 and list(m.ten_J_colind) == [0, 1, 2] and m.nJten == 3
  np.testing.assert_allclose(m.wrap_prm, [1, -0.5, 2])
  np.testing.assert_allclose(m.tendon_lengthspring[0], [0.1, 0.3])
  assert m.tendon_limited[0] and m.actuator_trntype[0] == 3
  J = np.array([1, -0.5, 2.0])
  assert m.tendon_invweight0[0] > 0
  # springlength -1 rests at the qpos0 length
  m2 = _model(ten='stiffness="10"')
  np.testing.assert_allclose(m2.tendon_lengthspring[0], [m2.tendon_length0[0]] * 2)
  _ = J


def test_oracle_length_jacobian_velocity_moment():
  mjm = _model()
  rng = np.random.default_rng(0)
  qpos = rng.normal(size=(3, mjm.nq))
  qvel = rng.normal(size=(3, mjm.nv))
  od = _od(mjm, qpos, qvel)
  od.fwd_position()
  od.fwd_velocity()
  coef = np.array([1, -0.5, 2.0])
  np.testing.assert_allclose(od.ten_length[:, 0], qpos @ coef, rtol=1e-12)
  np.testing.assert_allclose(od.ten_J, np.tile(coef, (3, 1)), rtol=1e-12)
  np.testing.assert_allclose(od.ten_velocity[:, 0], qvel @ coef, rtol=1e-12)
  # tendon motor: length = gear L, moment = gear J (actuator 0); the joint motor (actuator 1) is unchanged
  np.testing.assert_allclose(od.actuator_length[:, 0], 2 * qpos @ coef, rtol=1e-12)
  np.testing.assert_allclose(od.actuator_moment.reshape(3, 2, 3)[:, 0], np.tile(2 * coef, (3, 1)), rtol=1e-12)
  np.testing.assert_allclose(od.actuator_velocity[:, 0], 2 * qvel @ coef, rtol=1e-12)


def test_oracle_armature_spring_damper():
  base = _model()
  mjm = _model(ten='stiffness="10" damping="3" springlength="0.1 0.3" armature=".05"')
  rng = np.random.default_rng(1)
  qpos = rng.normal(0, 0.3, size=(4, mjm.nq))
  qvel = rng.normal(size=(4, mjm.nv))
  a, b = _od(base, qpos, qvel), _od(mjm, qpos, qvel)
  for od in (a, b):
    od.fwd_position()
    od.fwd_velocity()
  J = np.array([1, -0.5, 2.0])
  dM = (b.qM - a.qM).reshape(4, 3, 3)
  # ancestor pattern of qM: a-b are one chain, c is its own tree (no a-c / b-c coupling)
  want = 0.05 * np.outer(J, J)
  want[2, :2] = want[:2, 2] = 0.0
  np.testing.assert_allclose(dM, np.broadcast_to(want, dM.shape), atol=1e-12)
  L = qpos @ J
  fs = np.where(L > 0.3, 10 * (0.3 - L), np.where(L < 0.1, 10 * (0.1 - L), 0.0))
  np.testing.assert_allclose(b.qfrc_spring, fs[:, None] * J, atol=1e-12)
  np.testing.assert_allclose(b.qfrc_damper, (-3 * (qvel @ J))[:, None] * J, atol=1e-12)
  assert (L > 0.3).any() or (L < 0.1).any()


def test_oracle_limit_row_holds_the_range():
  """A tendon pushed by its motor against range [-.2, .2] comes to rest at the limit (soft), the
  LIMIT_TENDON row has J = -ten_J at the upper side."""
  mjm = _model(ten='range="-0.2 0.2"')
  od = _od(mjm, np.zeros((1, mjm.nq)), np.zeros((1, mjm.nv)), ctrl=np.array([[1.0, 0.0]]))
  for _ in range(2000):
    od.step()
  od.forward()
  L = float(od.ten_length[0, 0])
  assert 0.19 < L < 0.21, L
  n = int(od.nefc[0, 0])
  assert n == 1 and od.efc_type[0, 0] == 4 and int(od.nl[0, 0]) == 1
  np.testing.assert_allclose(od.efc_J[0, :3], -np.array([1, -0.5, 2.0]), atol=1e-12)
  assert abs(float(od.ten_velocity[0, 0])) < 1e-3  # at rest along the tendon (the null space may drift)


def test_oracle_friction_row_and_actuator_range():
  """frictionloss holds the tendon against a push below it (FRICTION_TENDON row, nf = 1); the tendon's
  actuatorfrcrange scales the motor force down to the range."""
  mjm = _model(ten='frictionloss="5" actuatorfrclimited="true" actuatorfrcrange="-1 1"')
  od = _od(mjm, np.zeros((1, mjm.nq)), np.zeros((1, mjm.nv)), ctrl=np.array([[3.0, 0.0]]))
  od.forward()
  assert int(od.nf[0, 0]) == 1 and od.efc_type[0, 0] == 2
  np.testing.assert_allclose(od.efc_frictionloss[0, 0], 5.0)
  np.testing.assert_allclose(od.actuator_force[0, 0], 1.0)  # gain 1 * ctrl 3 clamped by the tendon range
  free = _od(_model(ten='actuatorfrclimited="true" actuatorfrcrange="-1 1"'), np.zeros((1, mjm.nq)), np.zeros((1, mjm.nv)),
             ctrl=np.array([[3.0, 0.0]]))
  for _ in range(200):
    od.step()
    free.step()
  # the push 2 * 1 along the tendon (gear 2) is below the friction loss 5: the (soft) friction row holds
  # the tendon to a slow creep, 50x slower than without it, at a force inside [-5, 5]
  assert abs(float(od.ten_velocity[0, 0])) < abs(float(free.ten_velocity[0, 0])) / 50
  assert abs(float(od.efc_force[0, 0])) <= 5.0 + 1e-9


@pytest.mark.gpu
@pytest.mark.parametrize("solver", ["CG", "NEWTON"])
def test_gpu_tendon_matches_oracle(solver):
  import torch

  import mujoco_warp_amd as mjw

  mjm = _model(g=-9.81, ja='range="-1 1" limited="true"',
               ten='stiffness="10" damping="1" springlength="0 .2" range="-.3 .3" frictionloss=".3" armature=".05" '
                   'actuatorfrclimited="true" actuatorfrcrange="-2 2"')
  mjm.opt.solver = {"CG": 1, "NEWTON": 2}[solver]
  nworld = 16
  rng = np.random.default_rng(5)
  qpos = rng.normal(0, 0.4, (nworld, mjm.nq))
  qvel = rng.normal(0, 1.0, (nworld, mjm.nv))
  ctrl = rng.uniform(-2, 2, (nworld, mjm.nu))
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=16, nconmax=4)
  od = _od(mjm, qpos, qvel, ctrl)
  mjw.forward(m, d)
  od.forward()
  torch.cuda.synchronize()
  for f in ("ten_length", "ten_velocity", "actuator_length", "actuator_force", "qfrc_spring", "qfrc_damper", "qfrc_actuator",
            "qfrc_smooth"):
    want = getattr(od, f)
    np.testing.assert_allclose(np_(getattr(d, f)).reshape(want.shape), want, rtol=1e-5, atol=1e-6 * (np.abs(want).max() + 1), err_msg=f)
  np.testing.assert_allclose(np_(d.ten_J).reshape(od.ten_J.shape), od.ten_J, rtol=1e-6)
  np.testing.assert_allclose(np_(d.qM)[:, :3, :3].reshape(nworld, -1), od.qM, rtol=1e-5, atol=1e-7)
  for w in range(nworld):
    n = int(od.nefc[w, 0])
    assert int(d.nefc[w]) == n and (int(d.nf[w]), int(d.nl[w])) == (int(od.nf[w, 0]), int(od.nl[w, 0]))
    np.testing.assert_array_equal(d.efc.type[w, :n].cpu().numpy(), od.efc_type[w, :n])
    np.testing.assert_allclose(np_(d.efc.J[w, :n, :3]), od.efc_J[w].reshape(16, 3)[:n], rtol=1e-6, atol=1e-7)
    for f in ("pos", "vel", "D", "aref", "frictionloss"):
      np.testing.assert_allclose(np_(getattr(d.efc, f)[w, :n]), getattr(od, "efc_" + f)[w, :n], rtol=1e-4, atol=1e-5, err_msg=f)
  err = np.abs(np_(d.qacc) - od.qacc).max(axis=1) / (np.abs(od.qacc).max(axis=1) + 1)
  assert err.max() < 5e-3
  for _ in range(10):
    mjw.step(m, d)
    od.step()
  torch.cuda.synchronize()
  np.testing.assert_allclose(np_(d.qpos), od.qpos, rtol=2e-3, atol=2e-3)
