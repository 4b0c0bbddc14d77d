"""Connect / weld equality constraints (constraint.py:124-365, 792-1110), ball-joint limits
(:1421-1543) and their share of rne_postconstraint's cfrc_ext (smooth.py:1296-1430) -- SURVEY.md
§8(a) a14 / a26.

Oracle pinning (CPU): the compiler's qpos0 offsets make every connect / weld row zero at qpos0;
connect and weld translational rows are exact time derivatives (J qvel = d pos / dt, checked by
finite differences) and the rotational weld rows near the identity; a body connected to the world
swings about its anchor without drifting away; a welded body holds its pose under gravity; a ball
joint thrown past its cone limit is stopped near it.  `-m gpu`: rows, forces, sensors and a
rollout against the fp64 oracle on a model with every kind (body and site semantics).
"""

import numpy as np
import pytest

from tests.common import assert_close, gpu_from_state, np_, oracle_from_state

EQ_XML = """<mujoco><option timestep="0.002"/><worldbody>
<geom type="plane" size="5 5 .1"/>
<body name="a" pos="0 0 1"><freejoint/><geom type="box" size=".1 .05 .05"/><site name="sa" pos=".1 0 0"/></body>
<body name="b" pos=".2 0 1"><freejoint/><geom type="capsule" fromto="0 0 0 .2 0 0" size=".03"/><site name="sb" pos="-.1 0 0"/></body>
<body name="c" pos="-.5 0 1"><joint name="ball" type="ball" range="0 30" limited="true"/>
  <geom type="capsule" fromto="0 0 0 0 0 -.3" size=".03"/>
  <body name="c2" pos="0 0 -.3"><joint name="h" type="hinge" axis="1 0 0"/><geom type="sphere" size=".05"/></body>
</body>
<body name="d" pos="1 0 1"><freejoint/><geom type="sphere" size=".05"/><site name="sd" pos=".02 0 0"/></body>
<body name="e" pos="1.5 0 1"><freejoint/><geom type="box" size=".05 .05 .05"/></body>
</worldbody>
<equality>
<connect body1="a" anchor="0 0 .05"/>
<connect site1="sa" site2="sb"/>
<weld body1="d" anchor="1 0 1" torquescale="2"/>
<weld body1="e" body2="b" solref="0.01 1"/>
<joint joint1="h"/>
</equality>
<sensor><accelerometer site="sd"/><force site="sa"/><torque site="sd"/></sensor>
</mujoco>"""


def _model(xml=EQ_XML):
  from mujoco_warp_amd import mjcf

  return mjcf.load_model_from_string(xml)


def _states(mjm, nworld, seed, qnoise=0.02, vnoise=0.3):
  rng = np.random.default_rng(seed)
  qpos = np.tile(mjm.qpos0, (nworld, 1))
  for j in range(mjm.njnt):
    a = mjm.jnt_qposadr[j]
    if mjm.jnt_type[j] == 0:  # free: position + small rotation
      qpos[:, a : a + 3] += rng.normal(0, qnoise, (nworld, 3))
      q = qpos[:, a + 3 : a + 7] + rng.normal(0, qnoise, (nworld, 4))
      qpos[:, a + 3 : a + 7] = q / np.linalg.norm(q, axis=1, keepdims=True)
    elif mjm.jnt_type[j] == 1:
      q = qpos[:, a : a + 4] + rng.normal(0, 0.3, (nworld, 4))
      qpos[:, a : a + 4] = q / np.linalg.norm(q, axis=1, keepdims=True)
    else:
      qpos[:, a] += rng.normal(0, 0.1, nworld)
  qvel = rng.normal(0, vnoise, (nworld, mjm.nv))
  return qpos, qvel, np.zeros((nworld, mjm.nu))


def _rows(od, w, kind):
  ne = int(od.ne[w, 0])
  t = od.efc_id[w, :ne]
  return [r for r in range(ne) if od.om.mjm.eq_type[t[r]] == kind]


# ---- CPU: oracle / compiler pinning --------------------------------------------------------------
def test_compiler_offsets_zero_rows_at_qpos0():
  mjm = _model()
  assert list(mjm.eq_type) == [0, 0, 1, 1, 2] and list(mjm.eq_objtype) == [1, 6, 1, 1, 3]
  np.testing.assert_allclose(mjm.eq_data[0, 3:6], [0, 0, 1.05], atol=1e-12)  # anchor in the world frame
  om, od = oracle_from_state(mjm, mjm.qpos0[None], np.zeros((1, mjm.nv)), np.zeros((1, mjm.nu)))
  od.forward()
  assert int(od.ne[0, 0]) == 3 + 3 + 6 + 6 + 1
  np.testing.assert_allclose(od.efc_pos[0, :19], 0.0, atol=1e-12)


def _constraint_pos(mjm, qpos, qvel):
  om, od = oracle_from_state(mjm, qpos[None], qvel[None], np.zeros((1, mjm.nu)))
  od.fwd_position()
  return od


def test_connect_weld_jacobian_is_the_time_derivative():
  mjm = _model()
  qpos, qvel, _ = _states(mjm, 1, seed=1, qnoise=0.05, vnoise=1.0)
  od = _constraint_pos(mjm, qpos[0], qvel[0])
  J = od.efc_J[0].reshape(od.njmax, mjm.nv)
  h = 1e-7
  from oracle import orc  # noqa: F401  (oracle only: test infrastructure)

  def advance(q, v, dt):
    q = q.copy()
    for j in range(mjm.njnt):
      a, da, t = mjm.jnt_qposadr[j], mjm.jnt_dofadr[j], mjm.jnt_type[j]
      if t in (0, 1):
        lin = 3 if t == 0 else 0
        q[a : a + lin] += dt * v[da : da + lin]
        w = v[da + lin : da + lin + 3]
        quat = q[a + lin : a + lin + 4]
        ang = np.linalg.norm(w) * dt
        ax = w / max(np.linalg.norm(w), 1e-300)
        dq = np.r_[np.cos(ang / 2), np.sin(ang / 2) * ax]
        s0, u0, s1, u1 = quat[0], quat[1:], dq[0], dq[1:]
        qn = np.r_[s0 * s1 - u0 @ u1, s0 * u1 + s1 * u0 + np.cross(u0, u1)]  # quat * dq (local)
        q[a + lin : a + lin + 4] = qn / np.linalg.norm(qn)
      else:
        q[a] += dt * v[da]
    return q

  od2 = _constraint_pos(mjm, advance(qpos[0], qvel[0], h), qvel[0])
  fd = (od2.efc_pos[0] - od.efc_pos[0]) / h
  jv = J @ qvel[0]
  # connect rows 0..5 and weld translational rows: exact derivatives of p1 - p2
  for r in list(range(6)) + [6, 7, 8, 12, 13, 14]:
    assert abs(fd[r] - jv[r]) < 1e-5 * max(1.0, abs(jv[r])), (r, fd[r], jv[r])
  np.testing.assert_allclose(od.efc_vel[0, :19], jv[:19], atol=1e-12)


def test_connect_to_world_keeps_the_anchor():
  mjm = _model()
  om, od = oracle_from_state(mjm, mjm.qpos0[None], np.zeros((1, mjm.nv)), np.zeros((1, mjm.nu)))
  od.qvel[0, 3:6] = [2.0, 0.0, 0.0]  # spin body a about x
  for _ in range(300):
    od.step()
  xpos, R = od.xpos[0].reshape(-1, 3)[1], od.xmat[0].reshape(-1, 3, 3)[1]
  anchor = xpos + R @ np.array([0, 0, 0.05])
  assert np.linalg.norm(anchor - [0, 0, 1.05]) < 2e-3
  assert np.linalg.norm(xpos - [0, 0, 1.0]) > 1e-3  # it did swing
  # welded body d stays at its pose under gravity (soft-constraint sag only)
  assert np.linalg.norm(od.xpos[0].reshape(-1, 3)[5] - [1, 0, 1]) < 2e-3


def test_ball_limit_stops_the_cone():
  mjm = _model()
  om, od = oracle_from_state(mjm, mjm.qpos0[None], np.zeros((1, mjm.nv)), np.zeros((1, mjm.nu)))
  j = 2  # ball joint
  da, qa = mjm.jnt_dofadr[j], mjm.jnt_qposadr[j]
  od.qvel[0, da] = 6.0
  hit, peak = 0, 0.0
  for _ in range(200):
    od.step()
    hit += int(od.nl[0, 0])
    q = od.qpos[0, qa : qa + 4]
    peak = max(peak, 2 * np.arctan2(np.linalg.norm(q[1:]), q[0]))
  assert hit > 0
  # free flight would reach 6 rad/s * 0.4 s; the soft limit (solref 0.02) lets it overshoot a little
  assert np.deg2rad(30) < peak < np.deg2rad(30) + 0.1


def test_put_model_accepts_connect_weld_ball():
  import mujoco_warp_amd as mjw

  m = mjw.put_model(_model(), device="cpu")
  assert m.nlimited_ball == 1 and m.neq_cw == 4


# ---- GPU -------------------------------------------------------------------------------------------
@pytest.mark.gpu
def test_gpu_equality_rows_and_rollout_parity():
  import torch

  import mujoco_warp_amd as mjw

  mjm = _model()
  qpos, qvel, ctrl = _states(mjm, 32, seed=5)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=64, nconmax=16)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=64, nconmax=16)
  mjw.forward(m, d)
  od.forward()
  torch.cuda.synchronize()
  nv = mjm.nv
  for w in range(32):
    ne = int(od.ne[w, 0])
    assert int(d.ne[w]) == ne and int(d.nl[w]) == int(od.nl[w, 0])
    nl0 = ne + int(od.nf[w, 0])
    n = nl0 + int(od.nl[w, 0])
    np.testing.assert_array_equal(d.efc.type[w, :n].cpu().numpy(), od.efc_type[w, :n])
    np.testing.assert_array_equal(d.efc.id[w, :n].cpu().numpy(), od.efc_id[w, :n])
    assert_close(f"J[w{w}]", np_(d.efc.J[w, :n, :nv]), od.efc_J[w].reshape(od.njmax, nv)[:n], rtol=1e-4, atol=2e-5)
    for f in ("pos", "vel", "aref", "D"):
      assert_close(f"{f}[w{w}]", np_(getattr(d.efc, f)[w, :n]), getattr(od, "efc_" + f)[w, :n], rtol=1e-3, atol=1e-4)
  assert (od.nl[:, 0] > 0).any()  # some worlds start beyond the ball limit
  assert_close("qacc", np_(d.qacc), od.qacc, rtol=5e-3, atol=5e-2)
  assert_close("cfrc_ext", np_(d.cfrc_ext).reshape(32, -1), od.cfrc_ext, rtol=5e-3, atol=5e-2)
  assert_close("sensordata", np_(d.sensordata), od.sensordata, rtol=5e-3, atol=5e-2)
  m2, d2 = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=64, nconmax=16)
  om2, od2 = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=64, nconmax=16)
  for _ in range(10):
    mjw.step(m2, d2)
    od2.step()
  torch.cuda.synchronize()
  assert_close("qpos", np_(d2.qpos), od2.qpos, rtol=2e-3, atol=2e-3)
  assert_close("qvel", np_(d2.qvel), od2.qvel, rtol=2e-2, atol=2e-2)


@pytest.mark.gpu
def test_gpu_equality_generic_path_matches_dense():
  """njmax > 64 routes the step through the generic LDS kernel; same rows, same result."""
  import torch

  import mujoco_warp_amd as mjw

  mjm = _model()
  qpos, qvel, ctrl = _states(mjm, 8, seed=6)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=64, nconmax=16)
  m2, d2 = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=96, nconmax=16)
  mjw.forward(m, d)
  mjw.forward(m2, d2)
  torch.cuda.synchronize()
  for w in range(8):
    n = int(d.nefc[w])
    assert int(d2.nefc[w]) == n
    assert_close(f"J[w{w}]", np_(d2.efc.J[w, :n, : mjm.nv]), np_(d.efc.J[w, :n, : mjm.nv]), rtol=1e-5, atol=1e-6)
  assert_close("qacc", np_(d2.qacc), np_(d.qacc), rtol=5e-3, atol=5e-2)
