"""Every pair type of the reference's collision table (collision_driver.py:43-77, heightfields excluded) on
both device paths.

Primitive pairs run in the forward kernel's narrowphase (dense path) or the sparse collision kernel; the
multi-point / rare primitives (plane-ellipsoid, plane-cylinder, sphere-cylinder, plane-mesh) and every
CONVEX pair (GJK / EPA, box-box multi-contact; now with ellipsoids and cylinders too) run in the dense
path's pre-pass kernel (mjw_step.hip ccd_kernel) or the sparse path's CCD pre-pass.

CPU: the oracle on the MJCF scenes of the reference's collision_driver_test.py (tests/golden/
driver_fixtures.json, extracted as data) -- every scene yields contacts, as the reference asserts -- and
closed forms for the new primitives (plane-ellipsoid support depth, sphere-cylinder side / cap / rim).
GPU: the same scenes plus one seeded overlapping scene per convex pair type, on the dense and the sparse
path, contact for contact against the oracle.
"""

import json
import os

import numpy as np
import pytest

from tests.common import gpu_from_state, np_, oracle_from_state

HERE = os.path.dirname(os.path.abspath(__file__))
SCENES = json.load(open(os.path.join(HERE, "golden", "driver_fixtures.json")))["scenes"]

TYPES = {2: "sphere", 3: "capsule", 4: "ellipsoid", 5: "cylinder", 6: "box", 7: "mesh"}
SIZES = {2: ".12", 3: ".08 .12", 4: ".14 .09 .06", 5: ".1 .08", 6: ".1 .07 .05", 7: ""}
MESH = """<asset><mesh name="poly" vertex="0.12 0 0  0 0.1 0  -0.12 0 0  0 -0.1 0  0 0 0.14  0.02 0.01 -0.08"/></asset>"""
CONVEX = [(2, 4), (2, 7), (3, 4), (3, 5), (3, 7), (4, 4), (4, 5), (4, 6), (4, 7), (5, 5), (5, 6), (5, 7), (6, 6), (6, 7), (7, 7)]


def _geom(t):
  if t == 7:
    return '<geom type="mesh" mesh="poly"/>'
  return f'<geom type="{TYPES[t]}" size="{SIZES[t]}"/>'


def convex_scene(t1, t2):
  """Two free bodies with geoms of types t1 / t2, their centres 0.15 apart: every orientation overlaps
  (the smallest pair reaches 0.14) and most separate again within a few degrees."""
  return f"""<mujoco>{MESH}<option gravity="0 0 0"/><worldbody>
  <body pos="0 0 0"><freejoint/>{_geom(t1)}</body>
  <body pos="0.15 0.01 0.02"><freejoint/>{_geom(t2)}</body></worldbody></mujoco>"""


def _load(xml):
  from mujoco_warp_amd import mjcf

  return mjcf.load_model_from_string(xml)


def _oracle_contacts(mjm, qpos, nconmax=32):
  _, od = oracle_from_state(mjm, qpos, np.zeros((len(qpos), mjm.nv)), np.zeros((len(qpos), mjm.nu)), njmax=128, nconmax=nconmax)
  od.fwd_position()
  return od


@pytest.mark.parametrize("name", sorted(SCENES))
def test_oracle_driver_scenes_collide(name):
  """collision_driver_test.py:546-580 asserts contacts for every scene (against MuJoCo C)."""
  mjm = _load(SCENES[name])
  od = _oracle_contacts(mjm, mjm.qpos0[None])
  n = int(od.ncon[0, 0])
  assert n > 0
  assert np.all(np.isfinite(od.con_dist[0, :n])) and np.all(od.con_dist[0, :n] < 0)
  fr = od.con_frame[0, :9 * n].reshape(n, 3, 3)
  np.testing.assert_allclose(np.einsum("nij,nkj->nik", fr, fr), np.tile(np.eye(3), (n, 1, 1)), atol=1e-9)


def test_oracle_plane_ellipsoid_support_depth():
  """The deepest point of a rotated ellipsoid over a plane: depth = h - sqrt(n' R diag(s^2) R' n)."""
  from mujoco_warp_amd.mjcf import quat_to_mat

  s = np.array([0.1, 0.2, 0.3])
  rng = np.random.default_rng(0)
  for _ in range(5):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    h = 0.2
    xml = f"""<mujoco><worldbody><geom type="plane" size="5 5 .1"/><body pos="0 0 {h}" quat="{' '.join(map(str, q))}">
    <freejoint/><geom type="ellipsoid" size="{' '.join(map(str, s))}"/></body></worldbody></mujoco>"""
    mjm = _load(xml)
    od = _oracle_contacts(mjm, mjm.qpos0[None])
    R = quat_to_mat(q)
    reach = np.sqrt(np.array([0, 0, 1.0]) @ R @ np.diag(s * s) @ R.T @ np.array([0, 0, 1.0]))
    assert int(od.ncon[0, 0]) == (1 if h - reach < 0 else 0)
    if h - reach < 0:
      np.testing.assert_allclose(od.con_dist[0, 0], h - reach, rtol=1e-10)
      np.testing.assert_allclose(od.con_frame[0, :3], [0, 0, 1], atol=1e-12)


@pytest.mark.parametrize("where", ["side", "cap", "rim"])
def test_oracle_sphere_cylinder_closed_form(where):
  """Sphere (r .1) against an upright cylinder (r .15, half height .2): side = radial gap, cap = axial
  gap, rim = distance to the rim circle."""
  pos = {"side": (0.24, 0.0, 0.05), "cap": (0.03, 0.02, 0.29), "rim": (0.2, 0.0, 0.26)}[where]
  xml = f"""<mujoco><worldbody><body pos="{' '.join(map(str, pos))}"><freejoint/><geom type="sphere" size=".1"/></body>
  <geom type="cylinder" size=".15 .2"/></worldbody></mujoco>"""
  mjm = _load(xml)
  od = _oracle_contacts(mjm, mjm.qpos0[None])
  p = np.array(pos)
  if where == "side":
    want, n = np.hypot(p[0], p[1]) - 0.25, -np.array([p[0], p[1], 0]) / np.hypot(p[0], p[1])
  elif where == "cap":
    want, n = p[2] - 0.2 - 0.1, np.array([0, 0, -1.0])
  else:
    rim = np.array([0.15, 0, 0.2])
    want, n = np.linalg.norm(p - rim) - 0.1, (rim - p) / np.linalg.norm(p - rim)
  assert int(od.ncon[0, 0]) == 1
  np.testing.assert_allclose(od.con_dist[0, 0], want, rtol=1e-10)
  # the contact normal points from the sphere (geom 1 of the type-sorted pair) to the cylinder
  np.testing.assert_allclose(od.con_frame[0, :3], n, atol=1e-10)


def test_put_model_accepts_every_table_pair():
  import mujoco_warp_amd as mjw

  for t1, t2 in CONVEX:
    m = mjw.put_model(_load(convex_scene(t1, t2)), device="cpu")
    assert m.nxn_ccd == 1 and m.nxn_box == 1


# ---- GPU ------------------------------------------------------------------------------------------
def _match(mjm, d, od, w, tol_d, tol_p, tol_n):
  """Every oracle contact of world w found among the device's (same geoms, dist / pos / normal within the
  tolerances), and the counts equal."""
  n_or = int(od.ncon[w, 0])
  nacon = min(int(d.nacon[0]), d.naconmax)
  wid = d.contact.worldid[:nacon].cpu().numpy()
  sel = np.nonzero(wid == w)[0]
  assert len(sel) == n_or, (len(sel), n_or)
  gd, gp = np_(d.contact.dist[sel]), np_(d.contact.pos[sel])
  gf, gg = np_(d.contact.frame[sel]).reshape(-1, 9), d.contact.geom[sel].cpu().numpy()
  used = set()
  for i in range(n_or):
    og = sorted(od.con_geom[w, 2 * i:2 * i + 2])
    ok = [j for j in range(len(sel)) if j not in used and sorted(gg[j]) == og and abs(gd[j] - od.con_dist[w, i]) <= tol_d
          and np.abs(gp[j] - od.con_pos[w, 3 * i:3 * i + 3]).max() <= tol_p and np.abs(gf[j, :3] - od.con_frame[w, 9 * i:9 * i + 3]).max() <= tol_n]
    assert ok, (i, od.con_dist[w, i], od.con_pos[w, 3 * i:3 * i + 3], od.con_frame[w, 9 * i:9 * i + 3], gd, gp, gf[:, :3])
    used.add(ok[0])


def _gpu_vs_oracle(mjm, qpos, sparse, tol):
  import torch

  import mujoco_warp_amd as mjw

  if sparse:
    mjm.opt.jacobian = 1
  nworld = len(qpos)
  m, d = gpu_from_state(mjm, qpos, np.zeros((nworld, mjm.nv)), np.zeros((nworld, mjm.nu)), njmax=128, nconmax=16)
  assert bool(m.is_sparse) == sparse
  od = _oracle_contacts(mjm, qpos)
  mjw.fwd_position(m, d)
  torch.cuda.synchronize()
  for w in range(nworld):
    _match(mjm, d, od, w, *tol)


@pytest.mark.gpu
@pytest.mark.parametrize("sparse", [False, True])
@pytest.mark.parametrize("name", sorted(SCENES))
def test_gpu_driver_scenes_match_oracle(name, sparse):
  mjm = _load(SCENES[name])
  convex = any(k in name for k in ("box_box", "convex", "mesh"))
  tol = (2e-5, 2e-4, 2e-4) if convex else (2e-6, 2e-6, 2e-6)
  _gpu_vs_oracle(mjm, np.tile(mjm.qpos0, (2, 1)), sparse, tol)


@pytest.mark.gpu
@pytest.mark.parametrize("sparse", [False, True])
@pytest.mark.parametrize("pair", CONVEX, ids=[f"{TYPES[a]}-{TYPES[b]}" for a, b in CONVEX])
def test_gpu_convex_pairs_match_oracle(pair, sparse):
  """GJK / EPA of every convex pair type at 16 seeded orientations (overlapping or separated)."""
  mjm = _load(convex_scene(*pair))
  rng = np.random.default_rng(11)
  qpos = np.tile(mjm.qpos0, (16, 1))
  for b in range(2):
    q = rng.normal(size=(16, 4))
    qpos[:, 7 * b + 3:7 * b + 7] = q / np.linalg.norm(q, axis=1, keepdims=True)
  od = _oracle_contacts(mjm, qpos)
  assert int(od.ncon.sum()) > 0  # some orientations collide
  # smooth supports (ellipsoid, cylinder): EPA's witness point / normal come off a polytope face whose choice
  # differs between fp32 and fp64 once depth has converged; the depth still agrees to ~1e-6.  The reference
  # accepts rtol 5e-2 / atol 1e-2 against MuJoCo C for these (collision_driver_test.py:567-569).
  tol = (2e-5, 2e-3, 5e-2) if (4 in pair or 5 in pair) else (2e-5, 2e-4, 2e-3)
  _gpu_vs_oracle(mjm, qpos, sparse, tol)
