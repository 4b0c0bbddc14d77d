"""Convex collision (GJK / EPA / box multi-contact) for box-box pairs: SURVEY.md §8(f) f1 (apollo's
hand plates and soles), the reference's default route for box-box (collision_driver.py:74,
collision_convex.py:701-890, collision_gjk.py).

CPU tests pin the oracle with analytic cases (face-face overlap -> the 4 corners of the overlap
rectangle at the mid-plane, margin -> one EPA contact, separated -> none, a box comes to rest on a
box); `-m gpu` tests compare the HIP pre-pass + forward kernel with the fp64 oracle.
"""

import numpy as np
import pytest

from tests.common import assert_close, gpu_from_state, np_, oracle_from_state


def _two_boxes(margin=0.0, pos=(0.05, 0.02, 0.19), euler="0 0 0"):
  from mujoco_warp_amd import mjcf

  xml = (f'<mujoco><worldbody><geom type="box" size=".1 .1 .1" margin="{margin / 2}"/>'
         f'<body pos="{pos[0]} {pos[1]} {pos[2]}" euler="{euler}"><freejoint/>'
         f'<geom type="box" size=".1 .1 .1" margin="{margin / 2}"/></body></worldbody></mujoco>')
  return mjcf.load_model_from_string(xml)


def _oracle_contacts(mjm):
  from oracle import orc

  od = orc.OracleData(orc.OracleModel(mjm), 1, 32, 16)
  od.fwd_position()
  n = od.ncon[0, 0]
  return n, od.con_dist[0, :n], od.con_pos[0, : 3 * n].reshape(n, 3), od.con_frame[0, : 9 * n].reshape(n, 3, 3)


def test_oracle_boxbox_face_face_four_corners():
  n, dist, pos, frame = _oracle_contacts(_two_boxes())
  assert n == 4
  np.testing.assert_allclose(dist, -0.01, atol=1e-9)
  np.testing.assert_allclose(frame[:, 0], np.tile([0, 0, 1], (4, 1)), atol=1e-9)  # geom1 -> geom2
  corners = sorted(map(tuple, np.round(pos, 9)))
  want = sorted((x, y, 0.095) for x in (-0.05, 0.1) for y in (-0.08, 0.1))
  np.testing.assert_allclose(corners, want, atol=1e-9)


def test_oracle_boxbox_margin_gives_one_epa_contact():
  n, dist, pos, frame = _oracle_contacts(_two_boxes(margin=0.002))
  assert n == 1  # multi-contact is off when the pair has a margin (collision_gjk.py:2336-2338)
  np.testing.assert_allclose(dist, -0.01, atol=1e-7)
  np.testing.assert_allclose(frame[0, 0], [0, 0, 1], atol=1e-6)
  assert -0.05 <= pos[0, 0] <= 0.1 and -0.08 <= pos[0, 1] <= 0.1 and abs(pos[0, 2] - 0.095) < 1e-6


def test_oracle_boxbox_separated_and_within_margin():
  n, *_ = _oracle_contacts(_two_boxes(pos=(0.05, 0.02, 0.205)))
  assert n == 0
  n, dist, _, _ = _oracle_contacts(_two_boxes(margin=0.01, pos=(0.05, 0.02, 0.205)))
  assert n == 1 and abs(dist[0] - 0.005) < 1e-6  # inside the margin: a contact at positive distance


def test_oracle_boxbox_yawed_face_face():
  """Top box yawed 30 deg: still face-face; the clipped octagon is pruned to its largest quad."""
  n, dist, pos, frame = _oracle_contacts(_two_boxes(pos=(0.03, 0.0, 0.195), euler="0 0 30"))
  assert n == 4
  np.testing.assert_allclose(dist, -0.005, atol=1e-9)
  np.testing.assert_allclose(pos[:, 2], 0.0975, atol=1e-9)
  c, s = np.cos(np.pi / 6), np.sin(np.pi / 6)
  local = (pos[:, :2] - [0.03, 0.0]) @ np.array([[c, -s], [s, c]])  # into the yawed box frame
  assert np.all(np.abs(pos[:, :2]) <= 0.1 + 1e-9) and np.all(np.abs(local) <= 0.1 + 1e-9)


def test_oracle_box_rests_on_box():
  from mujoco_warp_amd import mjcf
  from oracle import orc

  xml = ('<mujoco><option timestep="0.002"/><worldbody><geom type="plane" size="5 5 .1"/>'
         '<geom type="box" size=".2 .2 .1" pos="0 0 .1"/>'
         '<body pos=".02 -.03 .31" euler="0 0 20"><freejoint/><geom type="box" size=".1 .08 .1"/></body></worldbody></mujoco>')
  mjm = mjcf.load_model_from_string(xml)
  od = orc.OracleData(orc.OracleModel(mjm), 1, 64, 32)
  for _ in range(500):
    od.step()
  assert abs(od.qpos[0, 2] - 0.3) < 2e-3 and np.abs(od.qvel[0]).max() < 2e-2


def test_apollo_put_model_routes_box_pairs_through_ccd():
  import os

  import mujoco_warp_amd as mjw
  from tests.common import ROOT

  mjm = mjw.load_model(os.path.join(ROOT, "models", "apptronik_apollo", "scene_flat.xml"))
  m = mjw.put_model(mjm, device="cpu")
  assert m.nxn_ccd == 6 and m.ccd_epa_iterations == 16  # all convex pairs are box-box (collision_convex.py:1127)
  ids = m.nxn_ccdid.numpy()
  assert sorted(ids[ids >= 0].tolist()) == list(range(6))


# ---- GPU parity ------------------------------------------------------------------------------
STACK_XML = """<mujoco><option timestep="0.002"/><worldbody><geom type="plane" size="5 5 .1"/>
<body pos="0 0 .1"><freejoint/><geom type="box" size=".1 .1 .1" margin="{m}"/></body>
<body pos="0 0 .3"><freejoint/><geom type="box" size=".08 .12 .1" margin="{m}"/></body>
<body pos="0 0 .5"><freejoint/><geom type="box" size=".1 .06 .1" margin="{m}"/></body>
</worldbody></mujoco>"""


def stack_states(mjm, nworld, seed, tilt, overlap=0.006):
  """Three stacked boxes, random yaw (face-face) or random tilt (general orientation), slight overlap."""
  from mujoco_warp_amd.mjcf import quat_to_mat

  rng = np.random.default_rng(seed)
  qpos = np.tile(mjm.qpos0, (nworld, 1))
  for w in range(nworld):
    z = 0.0
    for b in range(3):
      yaw = rng.uniform(-np.pi, np.pi)
      q = np.array([np.cos(yaw / 2), 0, 0, np.sin(yaw / 2)])
      if tilt:
        q = q + rng.normal(0, tilt, 4)
        q /= np.linalg.norm(q)
      half = mjm.geom_size[1 + b]
      ext = np.abs(quat_to_mat(q) @ np.diag(half)).sum(axis=1)[2]
      z += ext - rng.uniform(0.0, overlap)
      qpos[w, 7 * b : 7 * b + 3] = [rng.uniform(-0.03, 0.03), rng.uniform(-0.03, 0.03), z]
      qpos[w, 7 * b + 3 : 7 * b + 7] = q
      z += ext
  qvel = rng.normal(0, 0.1, (nworld, mjm.nv))
  return qpos, qvel, np.zeros((nworld, 0))


def _check_face_face(mjm, qpos_w, key, pts, ref_pts):
  """Multi-contact points of a yawed face-face pair: same count as the oracle, all inside both faces.
  The reference prunes a clipped polygon of more than 4 vertices with a greedy quad search
  (collision_gjk.py:1337-1374) that stops at the first non-improving move, so near-equal quad areas
  (0.04 % apart in one of these worlds) let rounding pick another valid quad; the individual points
  are therefore not compared."""
  from mujoco_warp_amd.mjcf import quat_to_mat

  for g in key:
    b = mjm.geom_bodyid[g] - 1
    R = quat_to_mat(qpos_w[7 * b + 3 : 7 * b + 7])
    local = (pts - qpos_w[7 * b : 7 * b + 3]) @ R
    assert np.all(np.abs(local[:, :2]) <= mjm.geom_size[g][:2] + 1e-4), (g, local)
  assert len(pts) == len(ref_pts)


def _compare_contacts(mjm, d, od, nworld, pos_tol, nrm_tol, min_boxbox, qpos=None):
  nacon = int(d.nacon[0])
  wid = d.contact.worldid[:nacon].cpu().numpy()
  geom = d.contact.geom[:nacon].cpu().numpy()
  dist = np_(d.contact.dist[:nacon])
  pos = np_(d.contact.pos[:nacon])
  frame = np_(d.contact.frame[:nacon]).reshape(-1, 9)
  nbb = 0
  for w in range(nworld):
    sel = np.nonzero(wid == w)[0]
    n = od.ncon[w, 0]
    og = od.con_geom[w, : 2 * n].reshape(n, 2)
    assert [tuple(x) for x in geom[sel]] == [tuple(x) for x in og], w
    assert_close(f"dist w{w}", dist[sel], od.con_dist[w, :n], rtol=1e-3, atol=2e-5)
    assert_close(f"normal w{w}", frame[sel, :3], od.con_frame[w, : 9 * n].reshape(n, 9)[:, :3], rtol=0, atol=nrm_tol)
    # points of one box-box pair come as a set (the quad pruning may start at another vertex)
    op = od.con_pos[w, : 3 * n].reshape(n, 3)
    for key in {tuple(x) for x in og}:
      i = [k for k in range(n) if tuple(og[k]) == key]
      boxbox = mjm.geom_type[key[0]] == 6 and mjm.geom_type[key[1]] == 6
      if boxbox and len(i) > 1:
        _check_face_face(mjm, qpos[w], key, pos[sel][i], op[i])
      else:
        assert_close(f"pos w{w} {key}", pos[sel][i], op[i], rtol=0, atol=pos_tol)
      nbb += boxbox
  assert nbb >= min_boxbox, nbb


@pytest.mark.gpu
def test_gpu_boxbox_face_face_multicontact():
  import torch

  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf

  mjm = mjcf.load_model_from_string(STACK_XML.format(m=0))
  nworld = 64
  qpos, qvel, ctrl = stack_states(mjm, nworld, seed=2, tilt=0.0)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=96, nconmax=24)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=96, nconmax=32)
  mjw.fwd_position(m, d)
  od.fwd_position()
  torch.cuda.synchronize()
  _compare_contacts(mjm, d, od, nworld, pos_tol=2e-4, nrm_tol=1e-4, min_boxbox=2 * nworld, qpos=qpos)


@pytest.mark.gpu
def test_gpu_boxbox_margin_epa_single_contact():
  import torch

  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf

  mjm = mjcf.load_model_from_string(STACK_XML.format(m=0.0005))
  nworld = 64
  qpos, qvel, ctrl = stack_states(mjm, nworld, seed=4, tilt=0.05, overlap=0.012)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=96, nconmax=24)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=96, nconmax=32)
  mjw.fwd_position(m, d)
  od.fwd_position()
  torch.cuda.synchronize()
  # EPA converges to ccd_tolerance (1e-6); fp32 vs fp64 witness points agree to ~1e-4
  _compare_contacts(mjm, d, od, nworld, pos_tol=2e-3, nrm_tol=2e-3, min_boxbox=nworld // 2, qpos=qpos)


@pytest.mark.gpu
def test_gpu_apollo_step_matches_oracle():
  import os

  import torch

  import mujoco_warp_amd as mjw
  from tests.common import ROOT

  mjm = mjw.load_model(os.path.join(ROOT, "models", "apptronik_apollo", "scene_flat.xml"))
  nworld = 32
  rng = np.random.default_rng(7)
  qpos = np.tile(mjm.key_qpos[0], (nworld, 1))
  qpos[:, 7:] += rng.normal(0, 0.05, (nworld, mjm.nq - 7))
  qvel = rng.normal(0, 0.2, (nworld, mjm.nv))
  ctrl = np.tile(mjm.key_ctrl[0], (nworld, 1))
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=64, nconmax=16)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=64, nconmax=16)
  for _ in range(3):
    mjw.step(m, d)
    od.step()
  torch.cuda.synchronize()
  assert np.isfinite(np_(d.qpos)).all()
  np.testing.assert_array_equal(d.nefc.cpu().numpy().reshape(-1), od.nefc.reshape(-1))
  from tests.test_gpu_parity_strict import normwise_close

  # normwise per world: qpos and the orientation sensor at the strict 1e-5, qvel at the reference's
  # Newton qacc bar carried through 3 steps (solver_test.py:32)
  normwise_close("qpos", np_(d.qpos), od.qpos)
  normwise_close("sensordata[quat]", np_(d.sensordata)[:, :4], od.sensordata[:, :4])
  normwise_close("qvel", np_(d.qvel), od.qvel, tol=5e-3)
