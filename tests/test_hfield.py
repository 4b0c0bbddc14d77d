"""Heightfield collisions (collision_convex.py:55-154 _hfield_filter, 158-697 ccd_hfield_kernel;
collision_gjk.py:178-187 prism support, 886-922 / 2160-2187 witness corrections), the six HFIELD entries of
the reference's collision table (collision_driver.py:50-55).

CPU: the compiler's <hfield> asset (normalised elevation, row-major grid) and geom; the oracle against the
reference's own known answers -- test_hfield_support (collision_gjk_test.py:811-880, the prism support
point for four directions, margin 0 and 0.1) and test_hfield_maxconpair (collision_driver_test.py:893-916:
a box over a 10 x 10 grid keeps 4 contacts out of the mjMAXCONPAIR-capped prism list) -- and closed forms:
a sphere over a flat and over a planar sloped heightfield (distance = signed plane distance - radius,
normal = the plane normal).  Contact sets beyond these are parity unpinned against MuJoCo C (not here).
GPU: the dense and the sparse pre-pass against the oracle, contact for contact, for every convex geom
type over a bumpy heightfield, and a short falling-box rollout.
"""

import numpy as np
import pytest

from tests.common import gpu_from_state, np_, oracle_from_state


def _load(xml):
  from mujoco_warp_amd import mjcf

  return mjcf.load_model_from_string(xml)


def test_compile_hfield_asset_and_geom():
  mjm = _load("""<mujoco><asset><hfield name="t" nrow="2" ncol="3" size="1 .5 .2 .1" elevation="1 3 2 5 4 7"/>
  <hfield name="flat" nrow="2" ncol="2" size=".3 .3 .1 .05"/></asset>
  <worldbody><geom type="hfield" hfield="flat"/><geom type="hfield" hfield="t" pos="2 0 0"/>
  <body pos="0 0 1"><freejoint/><geom type="sphere" size=".1"/></body></worldbody></mujoco>""")
  assert mjm.nhfield == 2 and mjm.nhfielddata == 10
  np.testing.assert_array_equal(mjm.hfield_nrow, [2, 2])
  np.testing.assert_array_equal(mjm.hfield_ncol, [3, 2])
  np.testing.assert_array_equal(mjm.hfield_adr, [0, 6])
  np.testing.assert_allclose(mjm.hfield_data[:6], (np.array([1, 3, 2, 5, 4, 7]) - 1) / 6.0)  # normalised to [0, 1]
  np.testing.assert_allclose(mjm.hfield_data[6:], 0.0)
  np.testing.assert_allclose(mjm.hfield_size, [[1, .5, .2, .1], [.3, .3, .1, .05]])
  np.testing.assert_array_equal(mjm.geom_type[:2], [1, 1])
  np.testing.assert_array_equal(mjm.geom_dataid[:3], [1, 0, -1])
  assert mjm.body_mass[0] == 0.0
  import mujoco_warp_amd as mjw

  m = mjw.put_model(mjm, device="cpu")
  assert m.nhfield == 2 and m.nhfielddata == 10
  assert m.nxn_ccd == 2  # both heightfields against the sphere take pre-pass slots


def test_compile_hfield_on_moving_body():
  """Heightfields may sit on moving bodies (the collision routines take the geom's frame).  MuJoCo's compiler
  gives a heightfield geom a box-like mass and inertia from its asset, which this compiler does not
  reproduce, so a moving body with a heightfield needs an explicit <inertial> (without one the model is
  refused).  (Image / binary heightfield files: tests/test_hfield_file.py.)"""
  mjm = _load(MOVING.format(elev=" ".join(["0"] * 42)))
  b = mjm.body_names.index("terrain")
  np.testing.assert_allclose(mjm.body_mass[b], 5.0)
  np.testing.assert_allclose(mjm.body_ipos[b], [0, 0, -0.3])
  assert int(mjm.geom_type[mjm.body_geomadr[b]]) == 1
  with pytest.raises(NotImplementedError, match="explicit <inertial>"):
    _load(MOVING.format(elev=" ".join(["0"] * 42)).replace(INERTIAL, ""))


# the bumpy heightfield of BUMPY on a free body of its own (plus a massive non-colliding box, whose mass and
# inertia the explicit <inertial> restates), a sphere on a second free body
INERTIAL = '<inertial pos="0 0 -.3" mass="5" diaginertia="0.0173333 0.0173333 0.0333333"/>'
MOVING = """<mujoco><option gravity="0 0 -9.81"/><asset>
<hfield name="h" nrow="6" ncol="7" size=".6 .5 .15 .1" elevation="{elev}"/></asset>
<worldbody>
<body name="terrain" pos=".05 -.03 0" euler="0 0 20"><freejoint/>{inertial}<geom type="hfield" hfield="h"/>
  <geom type="box" size=".1 .1 .02" pos="0 0 -.3" contype="0" conaffinity="0" mass="5"/></body>
<body pos="0 0 .2"><freejoint/><geom type="sphere" size=".12"/></body></worldbody></mujoco>""".replace("{inertial}", INERTIAL)


def _qmul(a, b):
  w1, x1, y1, z1 = a
  w2, x2, y2, z2 = b
  return np.array([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                   w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2, w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2])


def _qrot(q):
  w, x, y, z = q
  return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                   [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                   [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def _moving_worlds(mjm, nworld, seed=4):
  """World 0: the terrain at its default pose, the sphere somewhere over it; world k: both bodies moved by
  one rigid transform (R_k, t_k).  Returns qpos and the transforms."""
  rng = np.random.default_rng(seed)
  q0 = np.asarray(mjm.qpos0, np.float64).copy()
  q0[7:10] = [0.1, -0.05, 0.13]
  qpos, T = [q0], [(np.eye(3), np.zeros(3))]
  for _ in range(nworld - 1):
    qr = rng.normal(size=4)
    qr /= np.linalg.norm(qr)
    R, t = _qrot(qr), rng.uniform(-1, 1, 3)
    q = q0.copy()
    for a in (0, 7):
      q[a:a + 3] = R @ q0[a:a + 3] + t
      q[a + 3:a + 7] = _qmul(qr, q0[a + 3:a + 7])
    qpos.append(q)
    T.append((R, t))
  return np.stack(qpos), T


def test_oracle_moving_hfield_is_rigid_motion_invariant():
  """The same terrain-sphere configuration under rigid motions of both bodies: the same contact depths,
  the points and normals carried by the motion."""
  rng = np.random.default_rng(5)
  mjm = _load(MOVING.format(elev=" ".join(f"{v:.4f}" for v in rng.uniform(0, 1, 42))))
  qpos, T = _moving_worlds(mjm, 6)
  od = _oracle(mjm, qpos)
  n0, d0, p0, f0 = _contacts(od, 0)
  assert n0 >= 1
  for w in range(1, len(qpos)):
    n, d, p, f = _contacts(od, w)
    R, t = T[w]
    assert n == n0, w
    order = np.argsort(d0), np.argsort(d)
    np.testing.assert_allclose(d[order[1]], d0[order[0]], atol=1e-9)
    np.testing.assert_allclose(p[order[1]], (p0 @ R.T + t)[order[0]], atol=1e-7)
    np.testing.assert_allclose(f[order[1]], (f0 @ R.T)[order[0]], atol=1e-7)


@pytest.mark.parametrize("margin", [0.0, 0.1])
def test_oracle_hfield_support_kat(margin):
  """collision_gjk_test.py:811-880: bottom triangle at z = 0, top at 1 + margin; the geom's own margin 0."""
  from oracle import orc

  prism = np.array([[0, 0, 0], [1, 0, 0], [0.5, 1, 0], [0, 0, 1 + margin], [1, 0, 1 + margin], [0.5, 1, 1 + margin]])
  eps = 1e-3
  cases = [((eps, eps, 1.0), 5), ((-eps, -eps, -1.0), 0), ((1.0, eps, eps), 4), ((eps, 1.0, eps), 5)]
  for bits in (64, 32):
    for d, want in cases:
      pt, vi = orc.kat_hfield_support(prism, d, 0.0, real_bits=bits)
      np.testing.assert_allclose(pt, prism[want], rtol=1e-5)
      assert vi == (-2 if d[2] < 0 else -3)


MAXCONPAIR_XML = """<mujoco><asset><hfield name="hfield" nrow="10" ncol="10" size="1e-1 1e-1 1 1"/></asset>
<worldbody><body><joint type="slide" axis="0 0 1"/><geom type="box" size="1 1 .1"/></body>
<geom type="hfield" hfield="hfield"/></worldbody><keyframe><key qpos=".099"/></keyframe></mujoco>"""


def _oracle(mjm, qpos, nconmax=32, real_bits=64):
  _, od = oracle_from_state(mjm, qpos, np.zeros((len(qpos), mjm.nv)), np.zeros((len(qpos), mjm.nu)), njmax=256, nconmax=nconmax,
                            real_bits=real_bits)
  od.fwd_position()
  return od


def test_oracle_hfield_maxconpair():
  """collision_driver_test.py:893-916: nacon == 4 (the box covers 162 prisms, the list stops at 50)."""
  mjm = _load(MAXCONPAIR_XML)
  od = _oracle(mjm, np.array([[0.099]]))
  n = int(od.ncon[0, 0])
  assert n == 4
  np.testing.assert_allclose(od.con_dist[0, :n], -0.001, atol=1e-9)
  np.testing.assert_allclose(od.con_frame[0, :9 * n].reshape(n, 9)[:, :3], np.tile([0, 0, 1.0], (n, 1)), atol=1e-9)


def _sphere_scene(nrow, ncol, elevation, size, r=0.1):
  return f"""<mujoco><asset><hfield name="h" nrow="{nrow}" ncol="{ncol}" size="{size}" elevation="{elevation}"/></asset>
  <worldbody><geom type="hfield" hfield="h"/><body><freejoint/><geom type="sphere" size="{r}"/></body></worldbody></mujoco>"""


@pytest.mark.parametrize("sloped", [False, True])
def test_oracle_hfield_sphere_closed_form(sloped):
  """A planar heightfield -- flat, or rising linearly along x (the elevation of column c is c) -- under a
  sphere of radius 0.1: the deepest contact lies at the signed plane distance minus the radius, along the
  plane normal."""
  nrow, ncol, sx, sy, sz = 4, 5, 1.0, 0.8, 0.4
  elev = " ".join(str(float(c) if sloped else 0.0) for _ in range(nrow) for c in range(ncol))
  mjm = _load(_sphere_scene(nrow, ncol, elev, f"{sx} {sy} {sz} .2"))
  # z(x) = sz * (x + sx) / (2 sx) when sloped (normalised elevation c / (ncol - 1) at x = -sx + c dx), else 0
  slope = sz / (2 * sx) if sloped else 0.0
  nrm = np.array([-slope, 0.0, 1.0]) / np.hypot(slope, 1.0)
  rng = np.random.default_rng(3)
  qpos = np.tile(mjm.qpos0, (6, 1))
  for w in range(6):
    x, y = rng.uniform(-0.5, 0.5), rng.uniform(-0.4, 0.4)
    zs = slope * (x + sx) if sloped else 0.0
    qpos[w, :3] = [x, y, zs + rng.uniform(0.02, 0.09) / nrm[2]]  # penetrating by 0.01-0.08 along the normal
  od = _oracle(mjm, qpos)
  for w in range(6):
    n = int(od.ncon[w, 0])
    assert n >= 1
    c = qpos[w, :3]
    plane_dist = (c[2] - (slope * (c[0] + sx) if sloped else 0.0)) * nrm[2]
    d = od.con_dist[w, :n]
    np.testing.assert_allclose(d.min(), plane_dist - 0.1, atol=2e-6)
    k = int(np.argmin(d))
    np.testing.assert_allclose(od.con_frame[w, 9 * k:9 * k + 3], nrm, atol=2e-5)


BUMPY = """<mujoco>{mesh}<option gravity="0 0 -9.81"/><asset>
<hfield name="h" nrow="6" ncol="7" size=".6 .5 .15 .1" elevation="{elev}"/></asset>
<worldbody><geom type="hfield" hfield="h" pos=".05 -.03 0" euler="0 0 20"/>
<body pos="0 0 .2"><freejoint/>{geom}</body></worldbody></mujoco>"""
GEOMS = {
  "sphere": '<geom type="sphere" size=".12"/>',
  "capsule": '<geom type="capsule" size=".06 .12"/>',
  "ellipsoid": '<geom type="ellipsoid" size=".14 .09 .07"/>',
  "cylinder": '<geom type="cylinder" size=".1 .06"/>',
  "box": '<geom type="box" size=".12 .08 .05"/>',
  "mesh": '<geom type="mesh" mesh="poly"/>',
}
MESH = """<asset><mesh name="poly" vertex="0.12 0 0  0 0.1 0  -0.12 0 0  0 -0.1 0  0 0 0.09  0.02 0.01 -0.08"/></asset>"""


def bumpy_scene(kind):
  rng = np.random.default_rng(5)
  elev = " ".join(f"{v:.4f}" for v in rng.uniform(0, 1, 42))
  return BUMPY.format(mesh=MESH if kind == "mesh" else "", elev=elev, geom=GEOMS[kind])


def _bumpy_qpos(mjm, nworld, seed=11):
  rng = np.random.default_rng(seed)
  qpos = np.tile(mjm.qpos0, (nworld, 1))
  qpos[:, 0] = rng.uniform(-0.45, 0.45, nworld)
  qpos[:, 1] = rng.uniform(-0.35, 0.35, nworld)
  qpos[:, 2] = rng.uniform(0.1, 0.22, nworld)
  q = rng.normal(size=(nworld, 4))
  qpos[:, 3:7] = q / np.linalg.norm(q, axis=1, keepdims=True)
  return qpos


@pytest.mark.parametrize("kind", sorted(GEOMS))
def test_oracle_hfield_bumpy_contacts_sane(kind):
  """Every convex type over a rotated bumpy heightfield: contacts exist for most poses, each one with an
  orthonormal frame, a finite depth and a position inside the heightfield's footprint."""
  mjm = _load(bumpy_scene(kind))
  od = _oracle(mjm, _bumpy_qpos(mjm, 12))
  tot = 0
  for w in range(12):
    n = int(od.ncon[w, 0])
    tot += n
    assert n <= 4
    fr = od.con_frame[w, :9 * n].reshape(n, 3, 3)
    np.testing.assert_allclose(np.einsum("nij,nkj->nik", fr, fr), np.tile(np.eye(3), (n, 1, 1)), atol=1e-9)
    assert np.all(np.isfinite(od.con_dist[w, :n])) and np.all(od.con_dist[w, :n] < 0)
  assert tot >= 12


def _match(d, od, w, tol_d, tol_p, tol_n):
  n_or = int(od.ncon[w, 0])
  nacon = min(int(d.nacon[0]), d.naconmax)
  sel = np.nonzero(d.contact.worldid[:nacon].cpu().numpy() == w)[0]
  assert len(sel) == n_or, (w, len(sel), n_or)
  gd, gp, gf = np_(d.contact.dist[sel]), np_(d.contact.pos[sel]), np_(d.contact.frame[sel]).reshape(-1, 9)
  used = set()
  for i in range(n_or):
    ok = [j for j in range(len(sel)) if j not in used and abs(gd[j] - od.con_dist[w, i]) <= tol_d
          and np.abs(gp[j] - od.con_pos[w, 3 * i:3 * i + 3]).max() <= tol_p and np.abs(gf[j, :3] - od.con_frame[w, 9 * i:9 * i + 3]).max() <= tol_n]
    assert ok, (w, i, od.con_dist[w, i], od.con_pos[w, 3 * i:3 * i + 3], od.con_frame[w, 9 * i:9 * i + 3], gd, gp, gf[:, :3])
    used.add(ok[0])


def _contacts(od, w):
  n = int(od.ncon[w, 0])
  return n, od.con_dist[w, :n].copy(), od.con_pos[w, :3 * n].reshape(n, 3).copy(), od.con_frame[w, :9 * n].reshape(n, 9)[:, :3].copy()


def _same(a, b, tol_d, tol_p, tol_n):
  if a[0] != b[0]:
    return False
  used = set()
  for i in range(a[0]):
    ok = [j for j in range(b[0]) if j not in used and abs(a[1][i] - b[1][j]) <= tol_d and np.abs(a[2][i] - b[2][j]).max() <= tol_p
          and np.abs(a[3][i] - b[3][j]).max() <= tol_n]
    if not ok:
      return False
    used.add(ok[0])
  return True


def stable_worlds(mjm, qpos, tol, trials=9, eps=1e-6):
  """The worlds whose oracle contact set is well conditioned.  The reference's prism selection (the deepest,
  then the farthest points, with the 0 < d < 1e-3 duplicate cut) and its discrete EPA jump between answers at
  ties: a 1e-6 nudge of the pose can flip the set (as it flips between the fp32 and fp64 oracles), and two
  neighbouring prisms that return the bitwise-same witness (a shared vertex) pass the duplicate cut at
  d = 0 exactly, while any rounding difference (fp32 FMA contraction on the device) makes d tiny and cuts
  it.  Held to the oracle: the worlds whose set survives `trials` nudges of `eps` of the free joint's pose,
  each evaluated by the fp64 and the fp32 oracle, and holds no two points within 1e-3."""
  od = _oracle(mjm, qpos)
  rng = np.random.default_rng(1)
  stable = []
  for w in range(len(qpos)):
    ref = _contacts(od, w)
    ok = all(np.linalg.norm(ref[2][i] - ref[2][j]) >= 1e-3 for i in range(ref[0]) for j in range(i))
    for t in range(trials if ok else 0):
      q = qpos[w:w + 1].copy()
      if t:
        q[0, :7] += rng.normal(0, eps, 7)
        q[0, 3:7] /= np.linalg.norm(q[0, 3:7])
      if not all(_same(ref, _contacts(_oracle(mjm, q, real_bits=bits), 0), *tol) for bits in (64, 32)):
        ok = False
        break
    if ok:
      stable.append(w)
  return od, stable


@pytest.mark.gpu
@pytest.mark.parametrize("sparse", [False, True])
@pytest.mark.parametrize("kind", sorted(GEOMS))
def test_gpu_hfield_contacts_match_oracle(kind, sparse):
  import torch

  import mujoco_warp_amd as mjw

  mjm = _load(bumpy_scene(kind))
  if sparse:
    mjm.opt.jacobian = 1
  qpos = _bumpy_qpos(mjm, 16)
  m, d = gpu_from_state(mjm, qpos, np.zeros((16, mjm.nv)), np.zeros((16, mjm.nu)), njmax=256, nconmax=16)
  assert bool(m.is_sparse) == sparse
  # smooth supports (ellipsoid, cylinder): the fp32 / fp64 EPA face choice moves the witness point (cf.
  # test_collision_types.py), the depth agrees closely
  tol = (5e-5, 2e-3, 5e-2) if kind in ("ellipsoid", "cylinder") else (5e-5, 5e-4, 5e-3)
  od, stable = stable_worlds(mjm, qpos, tol)
  assert len(stable) >= 6, stable
  assert sum(int(od.ncon[w, 0]) for w in stable) > 0
  mjw.fwd_position(m, d)
  torch.cuda.synchronize()
  for w in stable:
    _match(d, od, w, *tol)


@pytest.mark.gpu
@pytest.mark.parametrize("sparse", [False, True])
def test_gpu_moving_hfield_matches_oracle(sparse):
  """The heightfield on a moving body: the device pre-pass reads its frame from the kinematics, as the oracle."""
  import torch

  import mujoco_warp_amd as mjw

  rng = np.random.default_rng(5)
  mjm = _load(MOVING.format(elev=" ".join(f"{v:.4f}" for v in rng.uniform(0, 1, 42))))
  if sparse:
    mjm.opt.jacobian = 1
  qpos, _ = _moving_worlds(mjm, 8)
  m, d = gpu_from_state(mjm, qpos, np.zeros((8, mjm.nv)), np.zeros((8, mjm.nu)), njmax=256, nconmax=16)
  assert bool(m.is_sparse) == sparse
  od = _oracle(mjm, qpos)
  mjw.fwd_position(m, d)
  torch.cuda.synchronize()
  for w in range(8):
    _match(d, od, w, 5e-5, 5e-4, 5e-3)


@pytest.mark.gpu
def test_gpu_hfield_maxconpair():
  """collision_driver_test.py:893-916 on the device: 4 contacts, depth 0.001."""
  import torch

  import mujoco_warp_amd as mjw

  mjm = _load(MAXCONPAIR_XML)
  m, d = gpu_from_state(mjm, np.array([[0.099]]), np.zeros((1, 1)), np.zeros((1, 0)), njmax=64, nconmax=16)
  mjw.fwd_position(m, d)
  torch.cuda.synchronize()
  assert int(d.nacon[0]) == 4
  np.testing.assert_allclose(np_(d.contact.dist[:4]), -0.001, atol=2e-6)


@pytest.mark.gpu
def test_gpu_hfield_sphere_rollout_matches_oracle():
  """Spheres rolling down the planar sloped heightfield of the closed-form test, started over the centroids
  of grid triangles (one deepest prism, no coincident witnesses): 30 Euler + CG steps, qpos against the
  fp64 oracle."""
  import torch

  import mujoco_warp_amd as mjw

  nrow, ncol, sx, sy, sz = 4, 5, 1.0, 0.8, 0.4
  elev = " ".join(str(float(c)) for _ in range(nrow) for c in range(ncol))
  mjm = _load(_sphere_scene(nrow, ncol, elev, f"{sx} {sy} {sz} .2"))
  slope = sz / (2 * sx)
  dx, dy = 2 * sx / (ncol - 1), 2 * sy / (nrow - 1)
  qpos = np.tile(mjm.qpos0, (4, 1))
  for w, (c, r, lower) in enumerate(((1, 0, True), (2, 1, False), (1, 1, True), (2, 0, False))):
    # the cell's two triangles: (c-1, r), (c, r), (c, r+1) style corners -- centroid of either half
    x0, y0 = -sx + dx * (c - 1), -sy + dy * r
    cx, cy = (x0 + dx * 2 / 3, y0 + dy / 3) if lower else (x0 + dx / 3, y0 + dy * 2 / 3)
    qpos[w, :3] = [cx, cy, slope * (cx + sx) + 0.098 * np.hypot(slope, 1.0)]
  m, d = gpu_from_state(mjm, qpos, np.zeros((4, mjm.nv)), np.zeros((4, mjm.nu)), njmax=64, nconmax=16)
  _, od = oracle_from_state(mjm, qpos, np.zeros((4, mjm.nv)), np.zeros((4, mjm.nu)), njmax=64, nconmax=16)
  for _ in range(30):
    mjw.step(m, d)
    od.step()
  torch.cuda.synchronize()
  np.testing.assert_allclose(np_(d.qpos), od.qpos, atol=1e-3)
  assert np.all(od.qpos[:, 0] < qpos[:, 0])  # rolled downhill (-x)
