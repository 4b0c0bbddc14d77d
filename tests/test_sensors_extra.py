"""Sensors past the frame / IMU set: touch (sensor.py:2001-2076), tendon position / velocity / actuator force,
joint and tendon limit position / velocity / force (sensor.py:243-278, 972-1007, 1538-1615), subtree linear
velocity and angular momentum (smooth.py:2932-3084) and potential / kinetic energy (sensor.py:2700-2940).

CPU: the oracle against closed forms -- tendon sensors are the tendon's length / velocity and its actuators'
force sum; limit sensors are the limit distance, J qvel and the limit row's force; the subtree linear velocity
is the time derivative of the subtree com; the angular momentum is sum(I w + m (x - c) x (v - v_c)); kinetic
energy is 1/2 qvel' M qvel; touch is the sum of the normal forces of the contacts whose normal ray meets the
site zone.  GPU: sensordata of the device against the oracle.
"""

import numpy as np
import pytest

from tests.common import gpu_from_state, np_, oracle_from_state

XML = """<mujoco><compiler angle="radian"/><option timestep="0.002"/>
<worldbody><geom type="plane" size="2 2 .1"/>
<body name="box" pos="0 0 .095"><freejoint/><geom type="box" size=".1 .1 .1" mass="1"/>
  <site name="touchall" type="box" size=".12 .12 .12"/><site name="touchtop" type="sphere" size=".02" pos="0 0 .1"/>
  <site name="touchcap" type="capsule" size=".03 .2" euler="0 90 0" pos="0 0 -.1"/></body>
<body name="arm" pos="1 0 1"><joint name="h1" type="hinge" axis="0 1 0" range="-.5 .5" limited="true"/>
  <geom type="capsule" fromto="0 0 0 .3 0 0" size=".03"/><site name="s1" pos=".3 0 0"/>
  <body pos=".3 0 0"><joint name="h2" type="hinge" axis="0 1 0" range="-1 1" limited="true" stiffness="3"/>
  <geom type="capsule" fromto="0 0 0 .3 0 0" size=".03"/><site name="s2" pos=".3 0 0"/></body></body>
</worldbody>
<tendon><fixed name="tf" limited="true" range="-.2 .2" stiffness="2" springlength=".05"><joint joint="h1" coef="1"/><joint joint="h2" coef="-1"/></fixed>
<spatial name="sp"><site site="s1"/><site site="s2"/></spatial></tendon>
<actuator><motor tendon="tf" gear="2"/><motor joint="h1"/><motor tendon="tf"/></actuator>
<sensor><touch site="touchall"/><touch site="touchtop"/><touch site="touchcap"/><tendonpos tendon="tf"/><tendonvel tendon="sp"/>
  <tendonactuatorfrc tendon="tf"/><jointlimitpos joint="h1"/><jointlimitvel joint="h1"/><jointlimitfrc joint="h1"/>
  <tendonlimitpos tendon="tf"/><tendonlimitvel tendon="tf"/><tendonlimitfrc tendon="tf"/><subtreelinvel body="arm"/>
  <subtreeangmom body="arm"/><subtreelinvel body="box"/><subtreeangmom body="world"/><e_potential/><e_kinetic/></sensor></mujoco>"""


def _model():
  from mujoco_warp_amd import mjcf

  return mjcf.load_model_from_string(XML)


def _state(mjm, nworld=4, seed=0):
  rng = np.random.default_rng(seed)
  qpos = np.tile(mjm.qpos0, (nworld, 1))
  qpos[:, 7] = 0.6 + 0.05 * rng.normal(size=nworld)  # h1 past its upper limit
  qpos[:, 8] = -0.3 + 0.1 * rng.normal(size=nworld)  # tendon h1 - h2 past its upper limit .2
  qvel = 0.3 * rng.normal(size=(nworld, mjm.nv))
  ctrl = rng.uniform(-1, 1, size=(nworld, mjm.nu))
  return qpos, qvel, ctrl


def _sens(mjm, od, w, k):
  a, n = mjm.sensor_adr[k], mjm.sensor_dim[k]
  return od.sensordata[w, a:a + n]


def test_oracle_tendon_limit_and_energy_sensors():
  mjm = _model()
  qpos, qvel, ctrl = _state(mjm)
  _, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=32, nconmax=8)
  od.forward()
  nv = mjm.nv
  for w in range(len(qpos)):
    L = od.ten_length[w]
    assert _sens(mjm, od, w, 3)[0] == L[0]
    assert _sens(mjm, od, w, 4)[0] == od.ten_velocity[w, 1]
    np.testing.assert_allclose(_sens(mjm, od, w, 5)[0], od.actuator_force[w, 0] + od.actuator_force[w, 2], rtol=1e-12)
    # joint h1 limit: distance to the upper limit, J qvel = -qvel, force of its row
    np.testing.assert_allclose(_sens(mjm, od, w, 6)[0], 0.5 - qpos[w, 7], atol=1e-12)
    np.testing.assert_allclose(_sens(mjm, od, w, 7)[0], -qvel[w, 6], atol=1e-12)
    rows = [r for r in range(int(od.nefc[w, 0])) if od.efc_type[w, r] == 3]
    assert len(rows) == 1 and _sens(mjm, od, w, 8)[0] == od.efc_force[w, rows[0]] >= 0
    # tendon limit: length h1 - h2 above .2
    np.testing.assert_allclose(_sens(mjm, od, w, 9)[0], 0.2 - L[0], atol=1e-12)
    assert L[0] > 0.2
    # energies
    M = od.qM[w].reshape(nv, nv)
    np.testing.assert_allclose(_sens(mjm, od, w, 17)[0], 0.5 * qvel[w] @ M @ qvel[w], rtol=1e-10)
    g = np.array(mjm.opt.gravity)
    xipos = od.xipos[w].reshape(-1, 3)
    pot = -sum(mjm.body_mass[b] * g @ xipos[b] for b in range(1, mjm.nbody))
    pot += 0.5 * 3 * (qpos[w, 8] - mjm.qpos_spring[8]) ** 2
    lo, hi = mjm.tendon_lengthspring[0]
    disp = hi - L[0] if L[0] > hi else (lo - L[0] if L[0] < lo else 0.0)
    pot += 0.5 * 2 * disp ** 2
    np.testing.assert_allclose(_sens(mjm, od, w, 16)[0], pot, rtol=1e-10)


def test_oracle_subtree_velocity_and_momentum():
  """subtreelinvel = d/dt subtree_com (central differences along qvel on the hinge arm; the free box's
  translational qvel is its com velocity); subtreeangmom(world) = sum over bodies of I w + m (x - c) x (v - v_c)."""
  mjm = _model()
  qpos, qvel, ctrl = _state(mjm, nworld=1)
  qvel[0, :6] = [0.1, -0.2, 0.3, 0.0, 0.0, 0.0]  # box: no spin, so its com velocity is qvel[:3]
  _, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=32, nconmax=8)
  od.forward()
  arm = mjm.body_names.index("arm")
  eps = 1e-6
  com = []
  for sgn in (1, -1):
    q = qpos.copy()
    q[0, 7:] += sgn * eps * qvel[0, 6:]
    _, o = oracle_from_state(mjm, q, qvel, ctrl, njmax=32, nconmax=8)
    o.fwd_position()
    com.append(o.subtree_com[0, 3 * arm:3 * arm + 3].copy())
  np.testing.assert_allclose(_sens(mjm, od, 0, 12), (com[0] - com[1]) / (2 * eps), atol=1e-7)
  np.testing.assert_allclose(_sens(mjm, od, 0, 14), qvel[0, :3], atol=1e-12)
  # total angular momentum about the world subtree com
  cvel = od.cvel[0].reshape(-1, 6)
  xipos, ximat = od.xipos[0].reshape(-1, 3), od.ximat[0].reshape(-1, 3, 3)
  c0 = od.subtree_com[0, :3]
  v = [cvel[b, 3:] - np.cross(xipos[b] - od.subtree_com[0, 3 * mjm.body_rootid[b]:3 * mjm.body_rootid[b] + 3], cvel[b, :3]) for b in range(mjm.nbody)]
  vc = sum(mjm.body_mass[b] * v[b] for b in range(mjm.nbody)) / mjm.body_subtreemass[0]
  Ltot = np.zeros(3)
  for b in range(1, mjm.nbody):
    R = ximat[b]
    Ltot += R @ (mjm.body_inertia[b] * (R.T @ cvel[b, :3])) + mjm.body_mass[b] * np.cross(xipos[b] - c0, v[b] - vc)
  np.testing.assert_allclose(_sens(mjm, od, 0, 15), Ltot, rtol=1e-9, atol=1e-12)


def test_oracle_touch_sensor_zones():
  """The box rests on the plane: the zone around the whole box sees every contact's normal force; the small
  sphere on top sees none; the capsule along the bottom face sees the contacts its ray meets."""
  mjm = _model()
  qpos, qvel, ctrl = _state(mjm, nworld=2)
  qvel[:] = 0
  _, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=32, nconmax=8)
  od.forward()
  for w in range(2):
    n = int(od.ncon[w, 0])
    assert n >= 4
    total = 0.0
    for c in range(n):
      adr = od.con_efc_address[w, 10 * c:10 * c + 10]
      total += sum(od.efc_force[w, adr[i]] for i in range(2 * (od.con_dim[w, c] - 1)))
    np.testing.assert_allclose(_sens(mjm, od, w, 0)[0], total, rtol=1e-12)
    assert _sens(mjm, od, w, 1)[0] == 0.0
    assert 0.0 <= _sens(mjm, od, w, 2)[0] <= total


@pytest.mark.gpu
@pytest.mark.parametrize("cone", [0, 1])
def test_gpu_extra_sensors_match_oracle(cone):
  import torch

  import mujoco_warp_amd as mjw

  mjm = _model()
  mjm.opt.cone = cone
  qpos, qvel, ctrl = _state(mjm, nworld=8, seed=3)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=32, nconmax=8)
  _, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=32, nconmax=8)
  mjw.forward(m, d)
  od.forward()
  torch.cuda.synchronize()
  got, want = np_(d.sensordata), od.sensordata
  for k in range(mjm.nsensor):
    a, n = mjm.sensor_adr[k], mjm.sensor_dim[k]
    scale = max(1.0, float(np.abs(want[:, a:a + n]).max()))
    # touch / limit forces come out of the solver (its bar: solver_test.py:32); the rest are kinematic
    tol = 5e-3 if mjm.sensor_type[k] in (0, 22, 25, 17) else 2e-5
    np.testing.assert_allclose(got[:, a:a + n], want[:, a:a + n], atol=tol * scale, err_msg=f"sensor {k} type {mjm.sensor_type[k]}")
