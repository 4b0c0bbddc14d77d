"""SURVEY.md §8(a) a26 + §8(f) f1 (config C4 apollo): sensors, rne_postconstraint, and the
sphere-box / capsule-box narrowphase.

CPU tests pin the oracle additions with analytic cases (a body welded to the world reads +g on its
accelerometer, a free-falling body reads 0, the force sensor of a hanging mass reads its weight,
...); `-m gpu` tests compare the HIP path with the fp64 oracle on seeded states.
"""

import os

import numpy as np
import pytest

from tests.common import ROOT, assert_close, gpu_from_state, np_, oracle_from_state

APOLLO = os.path.join(ROOT, "models", "apptronik_apollo", "scene_flat.xml")

# every supported sensor type, capsules / spheres / boxes on a floor; boxes do not touch boxes
SENSOR_XML = """<mujoco><option timestep="0.005"/>
<default><geom solref=".01 1"/></default>
<worldbody><geom name="floor" type="plane" size="5 5 .1"/>
 <site name="wsite" pos=".1 .2 .3" euler=".2 .1 .4"/>
 <body name="base" pos="0 0 .6"><freejoint/>
  <geom name="torso" type="box" size=".15 .1 .05" contype="2" conaffinity="1"/>
  <site name="imu" pos=".02 .01 .03" euler=".3 1.2 -.5"/>
  <body name="arm" pos=".15 0 0"><joint name="j1" axis="0 1 0" range="-1 1" damping=".5"/>
   <geom name="upper" type="capsule" fromto="0 0 0 .2 0 0" size=".03"/>
   <site name="tip" pos=".2 0 0"/>
   <body name="hand" pos=".2 0 0"><joint name="j2" axis="0 0 1" damping=".1"/><geom name="fist" type="sphere" size=".04"/></body>
  </body>
  <body name="leg" pos="-.1 0 -.05"><joint name="j3" axis="1 0 0" range="-.5 .5"/>
   <geom name="shin" type="capsule" fromto="0 0 0 0 0 -.3" size=".04"/>
   <body name="foot" pos="0 0 -.34"><joint name="j4" type="slide" axis="0 0 1" range="-.05 .05"/>
    <geom name="sole" type="box" size=".08 .05 .02" contype="2" conaffinity="1"/><site name="sole" pos="0 0 -.02"/>
   </body>
  </body>
 </body>
 <body name="ball" pos=".5 0 .3"><freejoint/><geom type="sphere" size=".06"/></body>
 <body name="rod" pos="-.5 0 .3"><freejoint/><geom type="capsule" size=".03 .1"/></body>
 <body name="crate" pos="0 .5 .2"><freejoint/><geom type="box" size=".1 .1 .1" contype="2" conaffinity="1"/></body>
</worldbody>
<actuator><motor name="m1" joint="j1" gear="10" ctrlrange="-1 1"/><position name="p3" joint="j3" kp="50" kv="2"/></actuator>
<sensor>
 <framequat objtype="site" objname="imu"/><gyro site="imu" cutoff="5"/><accelerometer site="imu" cutoff="100"/>
 <magnetometer site="imu"/><velocimeter site="tip"/><force site="sole"/><torque site="sole"/>
 <jointpos joint="j1"/><jointvel joint="j2"/><actuatorpos actuator="p3"/><actuatorvel actuator="p3"/>
 <actuatorfrc actuator="m1"/><jointactuatorfrc joint="j3"/>
 <framepos objtype="body" objname="hand" reftype="site" refname="imu"/><framepos objtype="xbody" objname="leg"/>
 <framexaxis objtype="geom" objname="upper"/><frameyaxis objtype="site" objname="tip" reftype="xbody" refname="base"/>
 <framezaxis objtype="body" objname="foot"/><framequat objtype="geom" objname="sole" reftype="body" refname="arm"/>
 <framelinvel objtype="site" objname="tip"/><framelinvel objtype="body" objname="hand" reftype="site" refname="imu"/>
 <frameangvel objtype="xbody" objname="arm" reftype="body" refname="leg"/><frameangvel objtype="geom" objname="fist"/>
 <framelinacc objtype="site" objname="tip"/><frameangacc objtype="body" objname="hand"/>
 <subtreecom body="base"/><clock/>
</sensor></mujoco>"""


def sensor_model():
  from mujoco_warp_amd import mjcf

  return mjcf.load_model_from_string(SENSOR_XML)


def sensor_states(mjm, nworld, seed=0):
  rng = np.random.default_rng(seed)
  qpos = np.tile(mjm.qpos0, (nworld, 1))
  for b in range(4):  # four free bodies: small random tilt, near the floor
    a = 7 * b
    q = np.array([1.0, 0, 0, 0]) + rng.normal(0, 0.3, (nworld, 4))
    qpos[:, a + 3 : a + 7] = q / np.linalg.norm(q, axis=1, keepdims=True)
    qpos[:, a + 2] = rng.uniform(0.02, 0.25, nworld) + (0.4 if b == 0 else 0.0)
  qpos[:, 7:11] += rng.normal(0, 0.3, (nworld, 4))  # j1 j2 j3 j4
  qpos[:, 10] = np.clip(qpos[:, 10], -0.05, 0.05)
  qvel = rng.normal(0, 0.5, (nworld, mjm.nv))
  ctrl = rng.uniform(-1, 1, (nworld, mjm.nu))
  return qpos, qvel, ctrl


# ---- host / compiler -------------------------------------------------------------------------
def test_apollo_compiles_with_imu_sensors():
  from mujoco_warp_amd import mjcf
  from mujoco_warp_amd.io import nxn_geom_pairs
  from mujoco_warp_amd.types import DataType, SensorType, Stage

  m = mjcf.load_model(APOLLO)
  # apptronik_apollo.xml: free base + 19 active hinges (the neck / wrist / shoulder_aa/ie joints are commented out)
  assert (m.nq, m.nv, m.nu, m.nsensor, m.nsensordata) == (26, 25, 19, 4, 13)
  assert m.sensor_type.tolist() == [SensorType.FRAMEQUAT, SensorType.GYRO, SensorType.ACCELEROMETER, SensorType.MAGNETOMETER]
  assert m.sensor_adr.tolist() == [0, 4, 7, 10] and m.sensor_dim.tolist() == [4, 3, 3, 3]
  assert m.sensor_needstage.tolist() == [Stage.POS, Stage.VEL, Stage.ACC, Stage.POS]
  assert m.sensor_datatype.tolist() == [DataType.QUATERNION, DataType.REAL, DataType.REAL, DataType.REAL]
  np.testing.assert_allclose(m.sensor_cutoff, [0, 54.9, 157, 0])
  assert m.opt.solver == 2 and m.opt.integrator == 0 and m.opt.disableflags & (1 << 15)
  pairs, _ = nxn_geom_pairs(m)
  kinds = sorted({tuple(sorted(m.geom_type[p])) for p in pairs})
  assert kinds == [(0, 3), (0, 6), (3, 3), (3, 6), (6, 6)]
  np.testing.assert_allclose(m.geom_margin[1:], 0.0005)


def test_sensor_model_put_model():
  import mujoco_warp_amd as mjw

  mjm = sensor_model()
  m = mjw.put_model(mjm, device="cpu")
  assert m.nsensor == 27 and m.sensor_rne_postconstraint == 1 and m.nsensor_acc == 7
  d = mjw.make_data(mjm, nworld=3, nconmax=16, njmax=64, device="cpu", m=m)
  assert tuple(d.sensordata.shape) == (3, mjm.nsensordata)


def test_unsupported_sensor_raises():
  from mujoco_warp_amd import mjcf

  with pytest.raises(NotImplementedError, match="rangefinder"):
    mjcf.load_model_from_string('<mujoco><worldbody><body><freejoint/><geom size=".1"/><site name="s"/></body></worldbody>'
                                '<sensor><rangefinder site="s"/></sensor></mujoco>')


# ---- oracle pinning (analytic) ---------------------------------------------------------------
def _single(xml, steps=0, **state):
  from mujoco_warp_amd import mjcf
  from oracle import orc

  mjm = mjcf.load_model_from_string(xml)
  od = orc.OracleData(orc.OracleModel(mjm), 1, 32, 16)
  for k, v in state.items():
    getattr(od, k)[0] = v
  for _ in range(steps):
    od.step()
  od.forward()
  return mjm, od


def test_oracle_welded_imu_reads_gravity_and_field():
  """A site on a body welded to the world: accelerometer = -g, gyro = 0, magnetometer = R^T B."""
  from mujoco_warp_amd.mjcf import quat_to_mat

  xml = ('<mujoco><option magnetic="0.1 -0.5 0.3"/><worldbody><body pos="0 0 1" euler="0.4 0.2 0.1">'
         '<geom size=".1" mass="2"/><site name="s" euler="1 .5 0.2"/></body></worldbody>'
         '<sensor><accelerometer site="s"/><gyro site="s"/><magnetometer site="s"/><framequat objtype="site" objname="s"/>'
         '<force site="s"/></sensor></mujoco>')
  mjm, od = _single(xml)
  q = od.sensordata[0, 9:13]
  R = quat_to_mat(q)
  np.testing.assert_allclose(od.sensordata[0, 0:3], R.T @ np.array([0, 0, 9.81]), atol=1e-12)
  np.testing.assert_allclose(od.sensordata[0, 3:6], 0, atol=1e-12)
  np.testing.assert_allclose(od.sensordata[0, 6:9], R.T @ np.array([0.1, -0.5, 0.3]), atol=1e-12)
  # force sensor of the welded 2 kg body: the parent holds its weight (cfrc_int, sensor.py:1483-1497)
  np.testing.assert_allclose(od.sensordata[0, 13:16], R.T @ np.array([0, 0, 2 * 9.81]), atol=1e-9)


def test_oracle_free_fall_accelerometer_reads_zero():
  xml = ('<mujoco><worldbody><body pos="0 0 5"><freejoint/><geom size=".1" contype="0" conaffinity="0"/>'
         '<site name="s" pos=".05 0 0"/></body></worldbody><sensor><accelerometer site="s"/><velocimeter site="s"/>'
         '<gyro site="s"/></sensor></mujoco>')
  _, od = _single(xml, steps=3, qvel=[0.1, 0.2, -0.3, 0, 0, 0])
  np.testing.assert_allclose(od.sensordata[0, 0:3], 0, atol=1e-9)
  v = np.array([0.1, 0.2, -0.3 - 9.81 * 0.002 * 3])
  np.testing.assert_allclose(od.sensordata[0, 3:6], v, atol=1e-9)
  np.testing.assert_allclose(od.sensordata[0, 6:9], 0, atol=1e-12)


def test_oracle_spinning_gyro_and_cutoff():
  """Hinge about z spinning at w: gyro = R^T (0,0,w) clamped by cutoff; framelinvel of an offset site = w x r."""
  xml = ('<mujoco><option gravity="0 0 0"/><worldbody><body><joint axis="0 0 1"/><geom size=".1" contype="0" conaffinity="0"/>'
         '<site name="s" pos=".3 0 0"/></body></worldbody><sensor><gyro site="s" cutoff="2"/><gyro site="s"/>'
         '<framelinvel objtype="site" objname="s"/><jointvel joint="0"/></sensor></mujoco>').replace('joint="0"', 'joint="j"').replace(
    '<joint axis', '<joint name="j" axis')
  _, od = _single(xml, qvel=[3.0])
  np.testing.assert_allclose(od.sensordata[0, 0:3], [0, 0, 2.0], atol=1e-12)  # clamped (REAL datatype)
  np.testing.assert_allclose(od.sensordata[0, 3:6], [0, 0, 3.0], atol=1e-12)
  np.testing.assert_allclose(od.sensordata[0, 6:9], [0, 0.9, 0], atol=1e-12)
  assert od.sensordata[0, 9] == 3.0


def test_oracle_sphere_box_and_capsule_box():
  """Sphere above a box face: dist = gap, normal = face normal; a capsule lying across the top face: 2 contacts."""
  from mujoco_warp_amd import mjcf
  from oracle import orc

  xml = ('<mujoco><worldbody><geom name="b" type="box" size=".2 .2 .1"/>'
         '<body pos=".05 -.03 .14"><freejoint/><geom type="sphere" size=".05"/></body>'
         '<body pos="0 .5 .2"><freejoint/><geom type="capsule" size=".02 .08" euler="0 90 0"/></body>'
         '<geom type="box" size=".3 .1 .1" pos="0 .5 0"/></worldbody></mujoco>')
  mjm = mjcf.load_model_from_string(xml)
  od = orc.OracleData(orc.OracleModel(mjm), 1, 32, 16)
  od.qpos[0, 2] = 0.14
  od.qpos[0, 9] = 0.119  # capsule axis along x, 1 mm into the top face (z = 0.1)
  od.fwd_position()
  n = od.ncon[0, 0]
  d = od.con_dist[0, :n]
  g = od.con_geom[0, : 2 * n].reshape(n, 2)
  frames = od.con_frame[0, : 9 * n].reshape(n, 3, 3)
  pos = od.con_pos[0, : 3 * n].reshape(n, 3)
  sph = [i for i in range(n) if mjm.geom_type[g[i, 0]] == 2]
  assert len(sph) == 1  # sphere-box (the other box is out of reach)
  i = sph[0]
  np.testing.assert_allclose(d[i], 0.14 - 0.1 - 0.05, atol=1e-12)
  np.testing.assert_allclose(frames[i, 0], [0, 0, -1], atol=1e-12)  # from sphere (geom1) into the box
  np.testing.assert_allclose(pos[i], [0.05, -0.03, 0.1 - 0.005], atol=1e-12)
  cap = [i for i in range(n) if mjm.geom_type[g[i, 0]] == 3]
  assert len(cap) == 2
  np.testing.assert_allclose(d[cap], -0.001, atol=1e-9)
  np.testing.assert_allclose(sorted(pos[cap][:, 0]), [-0.08, 0.08], atol=1e-9)


# ---- GPU parity ------------------------------------------------------------------------------
@pytest.mark.gpu
def test_gpu_sensors_match_oracle():
  import torch

  import mujoco_warp_amd as mjw

  mjm = sensor_model()
  nworld = 64
  qpos, qvel, ctrl = sensor_states(mjm, nworld, seed=3)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=64, nconmax=24)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=64, nconmax=64)
  mjw.forward(m, d)
  od.forward()
  torch.cuda.synchronize()
  got, want = np_(d.sensordata), od.sensordata
  # sensors that do not depend on the solver (position / velocity stage): smooth tolerance
  posvel = np.concatenate([np.arange(a, a + n) for a, n, st in zip(mjm.sensor_adr, mjm.sensor_dim, mjm.sensor_needstage) if st < 3])
  assert_close("pos/vel sensors", got[:, posvel], want[:, posvel], rtol=1e-4, atol=1e-4)
  np.testing.assert_array_equal(d.nefc.cpu().numpy().reshape(-1), od.nefc.reshape(-1))
  # acceleration sensors sit downstream of the iterative solver: relative to their scale
  acc = np.setdiff1d(np.arange(mjm.nsensordata), posvel)
  scale = np.abs(want[:, acc]).max(axis=0) + 1.0
  err = np.abs(got[:, acc] - want[:, acc]) / scale
  assert np.median(err) < 5e-3 and np.quantile(err, 0.95) < 5e-2, (np.median(err), np.quantile(err, 0.95))
  assert_close("cacc", np_(d.cacc), od.cacc.reshape(nworld, -1, 6), rtol=5e-2, atol=5e-2 * (1 + np.abs(od.cacc).max()))


@pytest.mark.gpu
def test_gpu_sensors_exact_inputs():
  """Acceleration sensors from the oracle's own qacc: isolates rne_postconstraint + sensor_acc from the solver."""
  import torch

  import mujoco_warp_amd as mjw

  mjm = sensor_model()
  mjm.opt.iterations = 0  # qacc = warmstart: identical inputs on both sides
  nworld = 32
  qpos, qvel, ctrl = sensor_states(mjm, nworld, seed=5)
  warm = np.random.default_rng(1).normal(0, 1, (nworld, mjm.nv))
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, qacc_warmstart=warm)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl, qacc_warmstart=warm)
  mjw.forward(m, d)
  od.forward()
  torch.cuda.synchronize()
  assert_close("qacc", np_(d.qacc), od.qacc, rtol=1e-5, atol=1e-5)
  assert_close("sensordata", np_(d.sensordata), od.sensordata, rtol=2e-4, atol=2e-3)
  # body forces: fp32 sums of terms up to ~1e6 here (random warmstart accelerations), so the absolute
  # tolerance scales with each world's largest entry
  for name, got, want in (("cfrc_int", np_(d.cfrc_int), od.cfrc_int), ("cfrc_ext", np_(d.cfrc_ext), od.cfrc_ext)):
    got = got.reshape(nworld, -1)
    scale = np.abs(want).max(axis=1, keepdims=True) + 1.0
    assert_close(name, got / scale, want / scale, rtol=0, atol=1e-5)


@pytest.mark.gpu
def test_gpu_box_contacts_match_oracle():
  import torch

  import mujoco_warp_amd as mjw

  mjm = sensor_model()
  nworld = 128
  qpos, qvel, ctrl = sensor_states(mjm, nworld, seed=11)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=64, nconmax=24)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl)
  mjw.fwd_position(m, d)
  od.fwd_position()
  torch.cuda.synchronize()
  nacon = int(d.nacon[0])
  wid = d.contact.worldid[:nacon].cpu().numpy()
  geom = d.contact.geom[:nacon].cpu().numpy()
  dist = np_(d.contact.dist[:nacon])
  pos = np_(d.contact.pos[:nacon])
  frame = np_(d.contact.frame[:nacon]).reshape(-1, 9)
  kinds = set()
  for w in range(nworld):
    sel = np.nonzero(wid == w)[0]
    n = od.ncon[w, 0]
    assert len(sel) == n, (w, len(sel), n)
    og = od.con_geom[w, : 2 * n].reshape(n, 2)
    key_o = [tuple(x) for x in og]
    key_g = [tuple(x) for x in geom[sel]]
    assert key_o == key_g  # same pairs, same order (pair order, then contact order)
    assert_close(f"dist w{w}", dist[sel], od.con_dist[w, :n], rtol=1e-3, atol=2e-5)
    assert_close(f"pos w{w}", pos[sel], od.con_pos[w, : 3 * n].reshape(n, 3), rtol=1e-3, atol=2e-5)
    assert_close(f"normal w{w}", frame[sel, :3], od.con_frame[w, : 9 * n].reshape(n, 9)[:, :3], rtol=1e-3, atol=1e-4)
    kinds |= {tuple(sorted(mjm.geom_type[list(k)])) for k in key_o}
  assert {(2, 6), (3, 6)} <= kinds, kinds  # both new narrowphase pairs were exercised
