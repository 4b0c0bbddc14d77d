"""Mesh geoms: the MJCF compiler's STL / OBJ loading and mesh inertia, mesh collisions on the sparse
path (GJK / EPA with mesh supports, collision_gjk.py:136-151; plane_convex,
collision_primitive.py:52-277) and the aloha_cloth benchmark scene (BASELINE.json C5) -- SURVEY.md
§8(f) f3.

Pinning without MuJoCo: a mesh that is a box must collide exactly like the analytic box, so the
oracle's mesh pairs are checked against its primitive sphere-box / plane-box / box-box results
(which are pinned by the box tests), and the compiler's mesh volume / inertia against the closed
form of a box.  `-m gpu`: the device against the fp64 oracle on the same scenes, and aloha_cloth
rollouts.
"""

import os
import struct

import numpy as np
import pytest

from tests.common import assert_close, gpu_from_state, np_, oracle_from_state

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ALOHA = os.path.join(ROOT, "models", "aloha_cloth", "scene.xml")

# unit cube [-1, 1]^3 as OBJ (quads, fan-triangulated by the loader; outward winding)
CUBE_OBJ = """v -1 -1 -1
v 1 -1 -1
v 1 1 -1
v -1 1 -1
v -1 -1 1
v 1 -1 1
v 1 1 1
v -1 1 1
f 1 4 3 2
f 5 6 7 8
f 1 2 6 5
f 2 3 7 6
f 3 4 8 7
f 4 1 5 8
"""
HALF = (0.1, 0.08, 0.06)


def _write_cube(tmp_path):
  (tmp_path / "cube.obj").write_text(CUBE_OBJ)
  # the same cube as a binary STL (12 triangles)
  v = np.array([[float(x) for x in ln.split()[1:]] for ln in CUBE_OBJ.splitlines() if ln.startswith("v")])
  quads = [[int(x) - 1 for x in ln.split()[1:]] for ln in CUBE_OBJ.splitlines() if ln.startswith("f")]
  tris = [t for q in quads for t in ((q[0], q[1], q[2]), (q[0], q[2], q[3]))]
  with open(tmp_path / "cube.stl", "wb") as f:
    f.write(b"\0" * 80 + struct.pack("<I", len(tris)))
    for t in tris:
      f.write(struct.pack("<3f", 0, 0, 0) + b"".join(struct.pack("<3f", *v[i]) for i in t) + b"\0\0")
  return tmp_path


def _scene(kind, tmp_path, file="cube.obj"):
  """Free `kind` geom (mesh cube / box) plus a free sphere and a plane; sparse path."""
  body = (f'<geom type="mesh" mesh="cube"/>' if kind == "mesh" else f'<geom type="box" size="{HALF[0]} {HALF[1]} {HALF[2]}"/>')
  xml = f"""<mujoco><compiler meshdir="."/><option jacobian="sparse" solver="CG" timestep="0.002"/>
<asset><mesh name="cube" file="{file}" scale="{HALF[0]} {HALF[1]} {HALF[2]}"/></asset>
<worldbody><geom type="plane" size="5 5 .1"/>
<body name="a" pos="0 0 .3"><freejoint/>{body}</body>
<body name="s" pos="0 0 .5"><freejoint/><geom type="sphere" size=".05"/></body>
<body name="b" pos=".5 0 .3"><freejoint/><geom type="box" size=".05 .05 .05"/></body>
</worldbody></mujoco>"""
  from mujoco_warp_amd import mjcf

  return mjcf.load_model_from_string(xml, basedir=str(tmp_path))


def _states(mjm, nworld, seed):
  """Cube tilted and lowered into the plane, sphere pressed onto the cube's top face, small box
  pressed into the cube's side (seeded per-world jitter)."""
  from mujoco_warp_amd.mjcf import quat_to_mat

  rng = np.random.default_rng(seed)
  qpos = np.tile(mjm.qpos0, (nworld, 1))
  for w in range(nworld):
    q = np.array([1.0, 0, 0, 0]) + rng.normal(0, 0.15, 4)
    q /= np.linalg.norm(q)
    R = quat_to_mat(q)
    low = np.abs(R @ np.diag(HALF)).sum(axis=1)[2]
    qpos[w, 0:3] = [0, 0, low - rng.uniform(0.002, 0.01)]
    qpos[w, 3:7] = q
    c = qpos[w, 0:3]
    top = c + R[:, 2] * HALF[2]  # top face centre, normal R[:, 2]
    qpos[w, 7:10] = top + R[:, 2] * (0.05 - rng.uniform(0.002, 0.01)) + R[:, 0] * rng.normal(0, 0.01)
    side = c + R[:, 0] * HALF[0]  # +x face centre
    qpos[w, 14:17] = side + R[:, 0] * (0.05 - rng.uniform(0.002, 0.008)) + R[:, 1] * rng.normal(0, 0.005)
  qvel = rng.normal(0, 0.1, (nworld, mjm.nv))
  return qpos, qvel, np.zeros((nworld, mjm.nu))


def _contacts(od, w):
  n = min(int(od.ncon[w, 0]), od.nconmax)
  out = []
  for c in range(n):
    out.append(dict(geom=tuple(int(x) for x in od.con_geom[w, 2 * c : 2 * c + 2]), dist=float(od.con_dist[w, c]),
                    pos=od.con_pos[w, 3 * c : 3 * c + 3].copy(), nrm=od.con_frame[w, 9 * c : 9 * c + 3].copy()))
  return out


# ---- CPU: compiler -------------------------------------------------------------------------------
def test_obj_and_stl_load_the_same_deduplicated_cube(tmp_path):
  from mujoco_warp_amd.mjcf import _read_mesh_file

  _write_cube(tmp_path)
  m_obj = _scene("mesh", tmp_path, "cube.obj")
  m_stl = _scene("mesh", tmp_path, "cube.stl")
  assert m_obj.nmesh == 1 and m_obj.mesh_vertnum[0] == 8 and m_stl.mesh_vertnum[0] == 8  # STL's 36 corners deduplicated
  np.testing.assert_allclose(np.sort(np.abs(m_obj.mesh_vert), axis=0), np.tile(HALF, (8, 1)))
  np.testing.assert_allclose(np.sort(m_obj.mesh_vert, axis=0), np.sort(m_stl.mesh_vert, axis=0))
  v, f = _read_mesh_file(str(tmp_path / "cube.obj"))
  assert v.shape == (8, 3) and f.shape == (12, 3)


def test_mesh_inertia_matches_the_box(tmp_path):
  _write_cube(tmp_path)
  mm, mb = _scene("mesh", tmp_path), _scene("box", tmp_path)
  np.testing.assert_allclose(mm.body_mass[1], mb.body_mass[1], rtol=1e-12)
  np.testing.assert_allclose(mm.body_mass[1], 1000 * 8 * np.prod(HALF), rtol=1e-12)
  np.testing.assert_allclose(np.sort(mm.body_inertia[1]), np.sort(mb.body_inertia[1]), rtol=1e-10)
  np.testing.assert_allclose(mm.body_ipos[1], 0.0, atol=1e-14)
  np.testing.assert_allclose(mm.geom_rbound[0 + 1], np.linalg.norm(HALF), rtol=1e-12)


def test_aloha_cloth_compiles():
  from mujoco_warp_amd import mjcf

  mjm = mjcf.load_model(ALOHA)
  assert mjm.nmesh == 25 and mjm.nflexvert == 900 and mjm.nu == 14 and mjm.nv == 16 + 2700
  # boundmass lifts the towel's 1.1e-4 kg vertices to 0.01 kg; the arms keep their inertials
  vb = mjm.flex_vertbodyid
  np.testing.assert_allclose(mjm.body_mass[vb], 0.01)
  assert abs(mjm.body_mass[2] - 0.969034) < 1e-9
  assert (mjm.geom_dataid[mjm.geom_type == 7] >= 0).all()


def test_put_model_routes_mesh_pairs_through_ccd():
  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf

  mjm = mjcf.load_model(ALOHA)
  m = mjw.put_model(mjm, device="cpu")
  assert m.is_sparse and m.nmesh == 25 and m.nxn_ccd > 0
  ccd = m.nxn_ccdid.numpy() >= 0
  kinds = {tuple(sorted((int(mjm.geom_type[a]), int(mjm.geom_type[b])))) for a, b in m.nxn_geom_pair_filtered.numpy()[ccd]}
  assert kinds <= {(2, 7), (3, 7), (6, 7), (7, 7), (6, 6)}


# ---- CPU: oracle mesh collisions against the analytic box --------------------------------------
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_oracle_mesh_cube_collides_like_the_box(tmp_path, seed):
  _write_cube(tmp_path)
  res = {}
  for kind in ("mesh", "box"):
    mjm = _scene(kind, tmp_path)
    qpos, qvel, ctrl = _states(mjm, 1, seed)
    om, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=128, nconmax=32)
    od.fwd_position()
    res[kind] = _contacts(od, 0)
  by = {k: {} for k in res}
  for k, cons in res.items():
    for c in cons:
      by[k].setdefault(c["geom"], []).append(c)
  plane, cube, sphere, small = 0, 1, 2, 3
  # plane: plane_convex keeps the corners within 1e-3 of the deepest one (up to 4) -- exactly the
  # plane_box corners in that depth window
  pm = sorted(by["mesh"][(plane, cube)], key=lambda c: c["dist"])
  pb = sorted(by["box"][(plane, cube)], key=lambda c: c["dist"])
  pb = [c for c in pb if c["dist"] < pb[0]["dist"] + 1e-3][:4]
  assert len(pm) == len(pb) > 0
  for a, b in zip(pm, pb):
    assert abs(a["dist"] - b["dist"]) < 1e-9
    np.testing.assert_allclose(a["pos"], b["pos"], atol=1e-9)
  # sphere on the top face: GJK/EPA on the mesh vs the analytic sphere_box
  key_m = (sphere, cube) if (sphere, cube) in by["mesh"] else (cube, sphere)
  key_b = (sphere, cube) if (sphere, cube) in by["box"] else (cube, sphere)
  (a,), (b,) = by["mesh"][key_m], by["box"][key_b]
  assert abs(a["dist"] - b["dist"]) < 1e-6
  assert abs(abs(a["nrm"] @ b["nrm"]) - 1) < 1e-6
  # small box against the cube's side: mesh-box (single EPA contact) has the box-box depth
  km = [k for k in by["mesh"] if small in k and cube in k][0]
  kb = [k for k in by["box"] if small in k and cube in k][0]
  dm = by["mesh"][km][0]["dist"]
  db = min(c["dist"] for c in by["box"][kb])
  assert len(by["mesh"][km]) == 1 and abs(dm - db) < 1e-6


# ---- GPU ----------------------------------------------------------------------------------------
@pytest.mark.gpu
def test_gpu_mesh_contacts_and_rollout_match_oracle(tmp_path):
  import torch

  import mujoco_warp_amd as mjw

  _write_cube(tmp_path)
  mjm = _scene("mesh", tmp_path)
  nworld = 16
  qpos, qvel, ctrl = _states(mjm, nworld, seed=7)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=128, nconmax=32)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=128, nconmax=32)
  mjw.fwd_position(m, d)
  torch.cuda.synchronize()
  od.fwd_position()
  for w in range(nworld):
    start, cnt = (int(x) for x in d.ncon_world[w].cpu().numpy())
    assert cnt == int(od.ncon[w, 0])
    g = sorted((tuple(d.contact.geom[s].tolist()), float(d.contact.dist[s])) for s in range(start, start + cnt))
    o = sorted((c["geom"], c["dist"]) for c in _contacts(od, w))
    for (gg, gd), (og, odist) in zip(g, o):
      assert gg == og and abs(gd - odist) < 2e-5, (w, gg, gd, odist)
  m2, d2 = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=128, nconmax=32)
  om2, od2 = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=128, nconmax=32)
  for _ in range(20):
    mjw.step(m2, d2)
    od2.step()
  torch.cuda.synchronize()
  assert_close("qpos", np_(d2.qpos), od2.qpos, rtol=5e-3, atol=5e-3)


def test_inline_vertex_only_mesh_hull():
  """An inline <mesh vertex=...> without faces compiles to its convex hull (mjcf._hull_faces): a cube's
  8 corners give 12 outward triangles and the box's volume-integral mass; a tetrahedron 4 faces and
  volume 1/6."""
  from mujoco_warp_amd import mjcf

  cube = " ".join(f"{x} {y} {z}" for x in (-0.5, 0.5) for y in (-0.5, 0.5) for z in (-0.5, 0.5))
  tet = "0 0 0 1 0 0 0 1 0 0 0 1"
  xml = f"""<mujoco><asset><mesh name="c" vertex="{cube}"/><mesh name="t" vertex="{tet}"/></asset><worldbody>
<body><freejoint/><geom type="mesh" mesh="c" density="1000"/></body>
<body pos="2 0 0"><freejoint/><geom type="mesh" mesh="t" density="600"/></body></worldbody></mujoco>"""
  m = mjcf.load_model_from_string(xml)
  np.testing.assert_allclose(m.body_mass[1], 1000.0, rtol=1e-9)
  np.testing.assert_allclose(m.body_mass[2], 600.0 / 6.0, rtol=1e-9)
  np.testing.assert_allclose(m.body_inertia[1], [1000.0 / 6.0] * 3, rtol=1e-9)  # m (a^2 + b^2) / 12, a = b = 1
  v = np.array([float(x) for x in cube.split()]).reshape(-1, 3)
  f = mjcf._hull_faces(v)
  assert len(f) == 12
  c = v.mean(axis=0)
  for i, j, k in f:
    assert np.dot(np.cross(v[j] - v[i], v[k] - v[i]), v[i] - c) > 0
