"""franka (joint equality, position + general-affine actuators,
implicitfast, mesh geoms that do not collide, plane-capsule) and plane-box contacts.

CPU tests pin the oracle additions with analytic cases; `-m gpu` tests compare the HIP path with
the fp64 oracle on seeded states (same tolerances as tests/test_gpu_parity.py).
"""

import numpy as np
import pytest

from tests.common import BOXES_XML, assert_close, boxes_states, franka_model, franka_states, gpu_from_state, np_, oracle_from_state


# ---- host / compiler -------------------------------------------------------------------------
def test_franka_compiles_to_reference_sizes():
  from mujoco_warp_amd.io import nxn_geom_pairs

  m = franka_model()
  assert (m.nq, m.nv, m.nu, m.nbody, m.neq) == (9, 9, 8, 12, 1)
  assert m.opt.integrator == 3 and m.opt.disableflags & (1 << 15)  # implicitfast, eulerdamp off (scene.xml:6-8)
  pairs, _ = nxn_geom_pairs(m)
  # only the hand capsule and the two fingertip_pad_collision_4 boxes reach the floor
  assert sorted(tuple(m.geom_type[p]) for p in pairs) == [(0, 3), (0, 6), (0, 6)]
  np.testing.assert_allclose(m.eq_data[0, :5], [0, 1, 0, 0, 0])
  np.testing.assert_allclose(m.actuator_biasprm[0, :3], [0, -1000, -20])  # position kp=1000 kv=20 (panda.xml)
  assert m.actuator_forcelimited.all()


def test_franka_put_model_and_unsupported_pairs():
  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf

  m = mjw.put_model(franka_model(), device="cpu")
  assert m.neq == 1 and m.eq_data.shape == (1, 1, 11)
  d = mjw.make_data(franka_model(), nworld=2, nconmax=4, njmax=16, device="cpu", m=m)
  assert d.eq_active.tolist() == [[1], [1]]
  bb = mjcf.load_model_from_string('<mujoco><worldbody><body><freejoint/><geom type="box" size=".1 .1 .1"/></body>'
                                   '<body pos="0 0 1"><freejoint/><geom type="box" size=".1 .1 .1"/></body></worldbody></mujoco>')
  bb.opt.disableflags |= 1 << 17  # NATIVECCD off routes box-box to the primitive box_box, not built
  with pytest.raises(NotImplementedError, match="box-box"):
    mjw.put_model(bb, device="cpu")


# ---- oracle pinning --------------------------------------------------------------------------
def test_oracle_box_rests_on_four_corners():
  from mujoco_warp_amd import mjcf
  from oracle import orc

  xml = ('<mujoco><option timestep="0.002"/><worldbody><geom type="plane" size="5 5 .1"/>'
         '<body pos="0 0 0.099"><freejoint/><geom type="box" size=".1 .1 .1"/></body></worldbody></mujoco>')
  bm = mjcf.load_model_from_string(xml)
  od = orc.OracleData(orc.OracleModel(bm), 1, 32, 16)
  od.fwd_position()
  assert od.ncon[0, 0] == 4  # bottom corners only (margin 0)
  np.testing.assert_allclose(od.con_dist[0, :4], -0.001, atol=1e-12)
  np.testing.assert_allclose(od.con_pos[0, :12].reshape(4, 3)[:, 2], -0.0005, atol=1e-12)  # corner - n * dist / 2
  for _ in range(400):
    od.step()
  assert abs(od.qpos[0, 2] - 0.1) < 1e-3 and np.abs(od.qvel[0]).max() < 1e-3


def test_oracle_implicitfast_damping_is_exact():
  """One slide dof with damping b: implicitfast gives v' = v M / (M + dt b) (forward.py:494-510)."""
  from mujoco_warp_amd import mjcf
  from oracle import orc

  xml = ('<mujoco><option timestep="0.01" integrator="implicitfast" gravity="0 0 0"/><worldbody>'
         '<body><joint type="slide" axis="1 0 0" damping="3"/><geom type="sphere" size=".1" mass="2" contype="0" conaffinity="0"/>'
         '</body></worldbody></mujoco>')
  m = mjcf.load_model_from_string(xml)
  od = orc.OracleData(orc.OracleModel(m), 1, 4, 4)
  od.qvel[0, 0] = 1.5
  od.step()
  M = m.body_mass[1] + m.dof_armature[0]
  np.testing.assert_allclose(od.qvel[0, 0], 1.5 * M / (M + 0.01 * 3), rtol=1e-12)


def test_oracle_implicitfast_position_actuator_kv():
  """Position actuator kv enters the implicit matrix: qDeriv += -kv (derivative.py:36-107)."""
  from mujoco_warp_amd import mjcf
  from oracle import orc

  xml = ('<mujoco><option timestep="0.01" integrator="implicitfast" gravity="0 0 0"/><worldbody>'
         '<body><joint name="j" type="slide" axis="1 0 0"/><geom type="sphere" size=".1" mass="2" contype="0" conaffinity="0"/>'
         '</body></worldbody><actuator><position joint="j" kp="50" kv="4"/></actuator></mujoco>')
  m = mjcf.load_model_from_string(xml)
  od = orc.OracleData(orc.OracleModel(m), 1, 4, 4)
  od.qvel[0, 0] = 1.0
  od.ctrl[0, 0] = 0.0
  od.step()
  M = m.body_mass[1]
  qacc = (-4.0 * 1.0) / M  # force = kp (ctrl - q) - kv v at q = 0
  np.testing.assert_allclose(od.qvel[0, 0], 1.0 + 0.01 * M * qacc / (M + 0.01 * 4.0), rtol=1e-12)


def test_oracle_franka_equality_couples_fingers():
  mjm = franka_model()
  qpos, qvel, ctrl = franka_states(mjm, 4, seed=21)
  _, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=16, nconmax=8)
  od.forward()
  assert (od.ne[:, 0] == 1).all() and (od.efc_type[:, 0] == 0).all()
  J = od.efc_J.reshape(4, 16, 9)[:, 0]
  np.testing.assert_allclose(J[:, 7], 1.0)
  np.testing.assert_allclose(J[:, 8], -1.0)  # polycoef (0 1 0 0 0): d rhs / d q2 = 1
  for _ in range(100):
    od.step()
  assert np.isfinite(od.qpos).all()
  assert np.abs(od.qpos[:, 7] - od.qpos[:, 8]).max() < 2e-3


# ---- GPU parity ------------------------------------------------------------------------------
def _gpu(mjm, qpos, qvel, ctrl, njmax, nconmax):
  torch = pytest.importorskip("torch")
  if not torch.cuda.is_available():
    pytest.skip("no GPU")
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=njmax, nconmax=nconmax)
  _, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=njmax, nconmax=64)  # pool semantics: no per-world cap
  return m, d, od


@pytest.mark.gpu
def test_gpu_franka_forward():
  import torch

  import mujoco_warp_amd as mjw

  mjm = franka_model()
  qpos, qvel, ctrl = franka_states(mjm, 16, seed=22)
  m, d, od = _gpu(mjm, qpos, qvel, ctrl, 16, 4)
  mjw.forward(m, d)
  torch.cuda.synchronize()
  od.forward()
  nw, nv = 16, 9
  from tests.test_gpu_parity_strict import normwise_close, strict_close

  # the strict bar (tests/test_gpu_parity_strict.py): smooth outputs elementwise rtol 1e-5 with a
  # 1e-6 * scale floor; rows J strict, aref through the impedance curve at 3e-4; qacc at the
  # reference solver bar (solver_test.py:32)
  for name in ("xpos", "xquat", "cinert", "cdof", "actuator_force", "qfrc_actuator", "qfrc_passive", "qfrc_bias", "qfrc_smooth"):
    strict_close(name, np_(getattr(d, name)).reshape(nw, -1), getattr(od, name))
  assert np.array_equal(np_(d.ne).astype(int), od.ne[:, 0]) and np.array_equal(np_(d.nefc).astype(int), od.nefc[:, 0])
  for w in range(nw):
    n = int(d.nefc[w])
    if n == 0:
      continue
    strict_close(f"J[w{w}]", np_(d.efc.J[w, :n, :nv]).reshape(1, -1), od.efc_J[w].reshape(16, nv)[:n].reshape(1, -1))
    normwise_close(f"aref[w{w}]", np_(d.efc.aref[w, :n])[None], od.efc_aref[w, :n][None], tol=3e-4)
  normwise_close("qacc", np_(d.qacc), od.qacc, tol=5e-3)


@pytest.mark.gpu
def test_gpu_franka_implicitfast_rollout():
  import torch

  import mujoco_warp_amd as mjw

  mjm = franka_model()
  qpos, qvel, ctrl = franka_states(mjm, 16, seed=23, qvel_noise=0.1)
  m, d, od = _gpu(mjm, qpos, qvel, ctrl, 16, 4)
  for _ in range(10):
    mjw.step(m, d)
    od.step()
  torch.cuda.synchronize()
  from tests.test_gpu_parity_strict import normwise_close

  # normwise per world: qpos at the strict 1e-5, qvel at the solver bar (it carries 10 solves)
  normwise_close("qpos", np_(d.qpos), od.qpos)
  normwise_close("qvel", np_(d.qvel), od.qvel, tol=5e-3)


@pytest.mark.gpu
def test_gpu_plane_box_contacts_and_rollout():
  import torch

  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf

  mjm = mjcf.load_model_from_string(BOXES_XML)
  qpos, qvel, ctrl = boxes_states(mjm, 32, seed=24)
  m, d, od = _gpu(mjm, qpos, qvel, ctrl, 64, 24)
  mjw.fwd_position(m, d)
  torch.cuda.synchronize()
  od.fwd_position()
  nacon = int(d.nacon[0])
  gw = np_(d.contact.worldid[:nacon]).astype(int)
  for w in range(32):
    sel = np.nonzero(gw == w)[0]
    nco = int(od.ncon[w, 0])
    assert len(sel) == nco, f"world {w}: {len(sel)} contacts vs oracle {nco}"
    assert_close(f"dist[w{w}]", np.sort(np_(d.contact.dist[:nacon])[sel]), np.sort(od.con_dist[w, :nco]), rtol=1e-3, atol=2e-5)
    assert int(d.nefc[w]) == int(od.nefc[w, 0])
  assert (od.ncon[:, 0] > 0).all()
  m2, d2, od2 = _gpu(mjm, qpos, qvel, ctrl, 64, 24)
  for _ in range(20):
    mjw.step(m2, d2)
    od2.step()
  torch.cuda.synchronize()
  assert_close("qpos", np_(d2.qpos), od2.qpos, rtol=5e-3, atol=5e-3)
