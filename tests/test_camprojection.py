"""camprojection sensor (sensor.py:128-190, 524-529): the pixel coordinates of a site in a camera's image.

The oracle is pinned by known answers of the pinhole model (a point on the optical axis lands on the image
centre; a point at the fovy edge on the top / bottom image border; the focal / sensorsize branch scales with
the focal length) and by an independent numpy restatement of the reference's matrix chain
proj = image @ focal @ rotation @ translation; the device follows the oracle under `-m gpu`.  The sensor
test of the reference (sensor_test.py:215-216) uses a default camera (resolution 1 x 1, fovy 45) and a
cutoff of 0.001 on the second sensor, which clamps REAL data to +-cutoff; both are in XML below.
"""

import numpy as np
import pytest

from tests.common import gpu_from_state, np_, oracle_from_state

XML = """<mujoco><worldbody>
  <body name="cambody" pos="0.1 -0.2 0.3" euler="20 -10 30"><freejoint/><geom type="sphere" size=".05"/>
    <camera name="camera" pos="0 0 0.1"/>
    <camera name="wide" pos="0.05 0 0" euler="0 10 0" fovy="80" resolution="640 480"/>
    <camera name="lens" pos="0 0.05 0" resolution="320 240" sensorsize="0.0036 0.0027" focal="0.004 0.0042"/>
    <camera name="pixels" pos="0 0 0" resolution="200 100" sensorsize="0.002 0.001" focalpixel="150 160"/>
  </body>
  <body name="target" pos="0.3 0.1 -1.2"><freejoint/><geom type="sphere" size=".05"/>
    <site name="s0"/><site name="s1" pos="0.2 -0.1 0.1"/></body>
</worldbody>
<sensor>
  <camprojection camera="camera" site="s0"/>
  <camprojection camera="camera" site="s0" cutoff=".001"/>
  <camprojection camera="wide" site="s1"/>
  <camprojection camera="lens" site="s0"/>
  <camprojection camera="pixels" site="s1"/>
</sensor></mujoco>"""


def _load(xml=XML):
  from mujoco_warp_amd import mjcf

  return mjcf.load_model_from_string(xml)


def _reference_chain(mjm, site_xpos, cam_xpos, cam_xmat, cam):
  """sensor.py:143-190 restated with numpy matrices, fp64."""
  xpos, R = cam_xpos, cam_xmat.reshape(3, 3)
  T = np.array([[1, 0, 0, -xpos[0]], [0, 1, 0, -xpos[1]], [0, 0, 1, -xpos[2]], [0, 0, 0, 1.0]])
  Rot = np.eye(4)
  Rot[:3, :3] = R.T
  res = mjm.cam_resolution[cam]
  ss = mjm.cam_sensorsize[cam]
  intr = mjm.cam_intrinsic[cam]
  if ss[0] != 0 and ss[1] != 0:
    fx = intr[0] / (ss[0] + 1e-15) * res[0]
    fy = intr[1] / (ss[1] + 1e-15) * res[1]
  else:
    fx = fy = 0.5 / np.tan(mjm.cam_fovy[cam] * np.pi / 360.0) * res[1]
  Fo = np.array([[-fx, 0, 0, 0], [0, fy, 0, 0], [0, 0, 1.0, 0], [0, 0, 0, 0]])
  Im = np.array([[1, 0, 0.5 * res[0], 0], [0, 1, 0.5 * res[1], 0], [0, 0, 1.0, 0], [0, 0, 0, 0]])
  ph = Im @ Fo @ Rot @ T @ np.r_[site_xpos, 1.0]
  den = ph[2]
  if abs(den) < 1e-15:
    den = np.clip(den, -1e-15, 1e-15)
  return ph[:2] / den


def _states(mjm, nworld, seed=2):
  rng = np.random.default_rng(seed)
  qpos = np.tile(mjm.qpos0, (nworld, 1))
  for j in range(mjm.njnt):
    a = mjm.jnt_qposadr[j]
    qpos[1:, a:a + 3] += rng.normal(0, 0.1, (nworld - 1, 3))
    q = qpos[1:, a + 3:a + 7] + rng.normal(0, 0.1, (nworld - 1, 4))
    qpos[1:, a + 3:a + 7] = q / np.linalg.norm(q, axis=1, keepdims=True)
  return qpos


def test_compiler_camera_intrinsics():
  mjm = _load()
  np.testing.assert_array_equal(mjm.cam_resolution, [[1, 1], [640, 480], [320, 240], [200, 100]])
  np.testing.assert_allclose(mjm.cam_intrinsic[2], [0.004, 0.0042, 0, 0])
  # focalpixel -> length: 150 px / 200 px * 0.002 m, 160 / 100 * 0.001
  np.testing.assert_allclose(mjm.cam_intrinsic[3][:2], [0.0015, 0.0016])
  assert mjm.sensor_dim.tolist() == [2] * 5


def test_oracle_known_answers():
  """Optical axis -> image centre; a point at the half-fovy angle above the axis -> the top row."""
  mjm = _load("""<mujoco><worldbody><camera name="c" pos="0 0 0" fovy="60" resolution="100 80"/>
    <site name="axis" pos="0 0 -2"/><site name="edge" pos="0 0 -2"/></worldbody>
    <sensor><camprojection camera="c" site="axis"/><camprojection camera="c" site="edge"/></sensor></mujoco>""")
  # the camera looks along -z; put the second site at angle fovy / 2 above the axis (y up in the camera frame)
  mjm.site_pos[1] = [0.0, 2.0 * np.tan(np.radians(30.0)), -2.0]
  _, od = oracle_from_state(mjm, mjm.qpos0[None], np.zeros((1, mjm.nv)), np.zeros((1, mjm.nu)))
  od.forward()
  sd = od.sensordata[0]
  np.testing.assert_allclose(sd[:2], [50.0, 40.0], atol=1e-9)
  # fy = 0.5 / tan(30 deg) * 80; y_pix = (fy * y + 40 z) / z with z = -2: 40 - fy tan(30) = 40 - 40 = 0
  np.testing.assert_allclose(sd[2:4], [50.0, 0.0], atol=1e-9)


def test_oracle_matches_reference_matrix_chain():
  mjm = _load()
  qpos = _states(mjm, 5)
  _, od = oracle_from_state(mjm, qpos, np.zeros((5, mjm.nv)), np.zeros((5, mjm.nu)))
  od.forward()
  cams = [0, 0, 1, 2, 3]
  sites = [0, 0, 1, 0, 1]
  for w in range(5):
    sxp = od.site_xpos[w].reshape(-1, 3)
    cxp, cxm = od.cam_xpos[w].reshape(-1, 3), od.cam_xmat[w].reshape(-1, 9)
    for k, (c, s) in enumerate(zip(cams, sites)):
      want = _reference_chain(mjm, sxp[s], cxp[c], cxm[c], c)
      if k == 1:  # cutoff 0.001 clamps REAL data (sensor.py:54-110)
        want = np.clip(want, -0.001, 0.001)
      np.testing.assert_allclose(od.sensordata[w, 2 * k:2 * k + 2], want, rtol=1e-9, atol=1e-9)


@pytest.mark.gpu
def test_gpu_camprojection_matches_oracle():
  import torch

  import mujoco_warp_amd as mjw

  mjm = _load()
  nworld = 8
  qpos = _states(mjm, nworld)
  z = np.zeros((nworld, mjm.nv))
  u = np.zeros((nworld, mjm.nu))
  m, d = gpu_from_state(mjm, qpos, z, u)
  _, od = oracle_from_state(mjm, qpos, z, u)
  mjw.forward(m, d)
  od.forward()
  torch.cuda.synchronize()
  got, want = np_(d.sensordata), od.sensordata
  # pixel coordinates of up to ~1e3: fp32 through the camera frame and a division by depth
  np.testing.assert_allclose(got, want, rtol=2e-5, atol=2e-4)
  assert np.abs(want).max() > 10.0
