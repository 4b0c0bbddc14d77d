"""Mesh multi-contact (MULTICCD; collision_gjk.py:1403-1790, 1929-2150; collision_convex.py:809-842).

The compiler builds MuJoCo's mesh polygon data from each mesh's convex hull (mjcf._mesh_polygons: the hull's
coplanar triangles merged into one polygon, counter-clockwise about the outward normal, and the polygons of
every vertex).  Pins:

  * the reference's own known answer `test_mesh_mesh_ccd` (collision_gjk_test.py:470-488: two mesh cubes, the
    top one turned 40 degrees, 4 contacts) -- on the oracle through tests/test_golden.py, and on the device
    through the pipeline here;
  * a mesh cube behaves as the box of the same size: with MULTICCD, mesh-mesh and box-mesh pairs give the
    contact set of the box-box pair (itself pinned by the reference's box-box KATs) -- same count, depth and
    normal, and the same points as a set (the polygon a face starts at may differ, so the order may);
  * without MULTICCD a mesh pair keeps one contact (collision_convex.py:809), and with a margin it has one
    contact even with MULTICCD (collision_gjk.py:2336-2338, io.py:372-409 then rejects the model).
"""

import numpy as np
import pytest

from tests.common import gpu_from_state, np_, oracle_from_state

CUBE = "-1 -1 -1 1 -1 -1 1 1 -1 1 1 1 1 -1 1 -1 1 -1 -1 1 1 -1 -1 1"

# two stacked pairs per scene: (lower, upper) cubes as meshes or boxes, the upper one turned
SCENE = """<mujoco><option><flag multiccd="{flag}"/></option>
<asset><mesh name="cube" vertex="{cube}" scale=".1 .1 .1"/></asset>
<worldbody>
  <body pos="0 0 0"><geom {a}/></body>
  <body pos="0.02 0.1 0.199"><freejoint/><geom {b}/></body>
  <body pos="1 0 0"><geom {a}/></body>
  <body pos="1.03 -0.05 0.197" euler="0 0 25"><freejoint/><geom {b}/></body>
</worldbody></mujoco>"""
MESH = 'type="mesh" mesh="cube"'
BOX = 'type="box" size=".1 .1 .1"'


def _load(a, b, flag="enable"):
  from mujoco_warp_amd import mjcf

  return mjcf.load_model_from_string(SCENE.format(flag=flag, cube=CUBE, a=a, b=b))


def _states(mjm, nworld, seed=0, tilt=2e-4):
  """Shifted a little per world and tilted by `tilt` (default well inside the face-alignment tolerance, 0.0016
  rad, collision_gjk.py:34: multi-contact; tilt 0.02 tests the single-contact branch)."""
  rng = np.random.default_rng(seed)
  qpos = np.tile(mjm.qpos0, (nworld, 1))
  for j in range(mjm.njnt):
    a = mjm.jnt_qposadr[j]
    qpos[1:, a:a + 3] += rng.normal(0, 0.002, (nworld - 1, 3)) * np.array([1, 1, 0.2])
    q = qpos[1:, a + 3:a + 7] + rng.normal(0, tilt, (nworld - 1, 4))
    qpos[1:, a + 3:a + 7] = q / np.linalg.norm(q, axis=1, keepdims=True)
  return qpos


def _contacts(od, w):
  n = int(od.ncon[w, 0])
  geoms = od.con_geom[w].reshape(-1, 2)[:n]
  return n, od.con_dist[w][:n], od.con_pos[w].reshape(-1, 3)[:n], od.con_frame[w].reshape(-1, 9)[:n], geoms


def _oracle(mjm, qpos):
  nw = len(qpos)
  _, od = oracle_from_state(mjm, qpos, np.zeros((nw, mjm.nv)), np.zeros((nw, mjm.nu)), njmax=128, nconmax=32)
  od.fwd_position()
  return od


def _as_sets(pos):
  return sorted(tuple(np.round(p, 7)) for p in pos)


def _area4(a, b, c, d):
  """collision_gjk.py:1331-1334 _area4."""
  return 0.5 * np.linalg.norm(np.cross(a - d, d - b) + np.cross(b - c, c - a))


def _polygon_quad_run(P, tol, forced):
  """collision_gjk.py:1337-1374 _polygon_quad on the polygon P, in fp64, except that every comparison of two
  areas within `tol` of each other (a near-tie fp32 rounding may decide either way) takes its outcome from
  `forced` (then from the exact comparison, recorded).  Returns the kept quad and every near-tie outcome."""
  n = len(P)
  k = 0
  dec = list(forced)

  def grows(mn, m):  # the reference's `not (m_next <= m)`
    nonlocal k
    if abs(mn - m) > tol:
      return mn > m
    if k == len(dec):
      dec.append(bool(mn > m))
    k += 1
    return dec[k - 1]

  b, c, d = 1, 2, 3
  res = (0, b, c, d)
  m = _area4(P[0], P[b], P[c], P[d])
  for a in range(n):
    while True:
      mn = _area4(P[a], P[b], P[c], P[(d + 1) % n])
      if not grows(mn, m):
        break
      m, d = mn, (d + 1) % n
      res = (a, b, c, d)
      while True:
        mn = _area4(P[a], P[b], P[(c + 1) % n], P[d])
        if not grows(mn, m):
          break
        m, c = mn, (c + 1) % n
        res = (a, b, c, d)
      while True:
        mn = _area4(P[a], P[(b + 1) % n], P[c], P[d])
        if not grows(mn, m):
          break
        m, b = mn, (b + 1) % n
        res = (a, b, c, d)
    if b == a:
      b = (b + 1) % n
      if c == b:
        c = (c + 1) % n
        if d == c:
          d = (d + 1) % n
  return res, dec


def reachable_quads(P, rtol=1e-6):
  """Every quad _polygon_quad keeps on P when each near-equal area comparison (within rtol x the squared
  polygon diameter, far above fp32's error on these sums) may go either way."""
  P = np.asarray(P, np.float64)
  diam = max(np.linalg.norm(p - q) for p in P for q in P)
  tol = rtol * diam * diam
  out, seen, stack = set(), set(), [()]
  while stack:
    pre = stack.pop()
    if pre in seen:
      continue
    seen.add(pre)
    res, dec = _polygon_quad_run(P, tol, pre)
    out.add(res)
    for i in range(len(pre), len(dec)):
      stack.append(tuple(dec[:i]) + (not dec[i],))
  return out, len(seen) > 1


def turned_pair_candidates(mjm, qpos_w):
  """The fp64 oracle's contacts of the turned pair (x > 0.5) of one world, and the candidate contact sets
  the reference's greedy quad search can keep on its clipped polygon under fp32 rounding: each candidate
  is the quad's polygon vertices shifted like the oracle's own points (contact pos = vertex - dir / 2)."""
  od = _oracle(mjm, qpos_w[None])
  od2 = _oracle(mjm, qpos_w[None])
  polys = od2.fwd_position_polygons()
  _, _, pos, _, _ = _contacts(od, 0)
  mine = pos[pos[:, 0] > 0.5]
  polys = [(q, P) for q, P in polys if P[:, 0].mean() > 0.5]
  if not polys:  # the clipped polygon had at most 4 vertices: no search, one answer
    return mine, [mine], False
  assert len(polys) == 1, len(polys)
  q, P = polys[0]
  offset = mine.mean(axis=0) - P[list(q)].mean(axis=0)
  quads, tie = reachable_quads(P)
  assert tuple(int(i) for i in q) in quads
  return mine, [P[list(qq)] + offset for qq in sorted(quads)], tie


def same_points(a, b, tol=2e-4):
  a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
  return len(a) == len(b) and all(np.min(np.linalg.norm(b - p, axis=1)) < tol for p in a) and \
      all(np.min(np.linalg.norm(a - p, axis=1)) < tol for p in b)


def test_compiler_cube_polygons():
  from mujoco_warp_amd import mjcf

  mjm = _load(MESH, MESH)
  assert mjm.mesh_polynum.tolist() == [6] and mjm.mesh_polyvertnum.tolist() == [4] * 6
  assert mjm.mesh_polymapnum.tolist() == [3] * 8  # every corner of a cube lies on 3 faces
  v = np.asarray(mjm.mesh_vert).reshape(-1, 3)
  for k in range(6):
    loop = mjm.mesh_polyvert[mjm.mesh_polyvertadr[k]:mjm.mesh_polyvertadr[k] + 4]
    n = mjm.mesh_polynormal[k]
    assert abs(abs(n).max() - 1.0) < 1e-12  # axis-aligned unit normals
    c = np.cross(v[loop[1]] - v[loop[0]], v[loop[2]] - v[loop[0]])
    assert np.dot(c, n) > 0  # counter-clockwise about the outward normal
    assert np.allclose(v[loop] @ n, 0.1)  # every vertex on the face plane
  # a vertex off the hull (an interior point) maps to no polygon
  m2 = mjcf.load_model_from_string(f'<mujoco><asset><mesh name="c" vertex="{CUBE} 0 0 0.5"/></asset><worldbody><geom type="mesh" mesh="c"/></worldbody></mujoco>')
  assert m2.mesh_polymapnum[-1] == 0


@pytest.mark.parametrize("pair", ["mesh-mesh", "box-mesh", "mesh-box"])
def test_oracle_mesh_cube_equals_box(pair):
  a, b = {"mesh-mesh": (MESH, MESH), "box-mesh": (BOX, MESH), "mesh-box": (MESH, BOX)}[pair]
  mm, mb = _load(a, b), _load(BOX, BOX)
  qpos = _states(mm, 6)
  om, ob = _oracle(mm, qpos), _oracle(mb, qpos)
  total = 0
  for w in range(6):
    n1, d1, p1, f1, _ = _contacts(om, w)
    n2, d2, p2, f2, _ = _contacts(ob, w)
    assert n1 == n2, (w, n1, n2)
    total += n1
    np.testing.assert_allclose(np.sort(d1), np.sort(d2), atol=1e-9)
    # one normal per pair; the narrowphase orders a pair by geom type (box before mesh), so "mesh-box" has the
    # geoms, and the normal, the other way round
    # (EPA then resolves the other Minkowski difference: the normal of the other, tilt-1e-4 face)
    sgn = -1.0 if pair == "mesh-box" else 1.0
    np.testing.assert_allclose(sgn * f1[:, :3], f2[:, :3], atol=1e-9 if pair != "mesh-box" else 2e-3)
    # the first pair's clipped polygon is the 4-corner overlap rectangle: the same points; the turned pair's
    # is an 8-gon, of which polygon_quad keeps 4 starting from the polygon's first vertex, which depends on
    # where each face's loop starts -- there every point must lie in the overlap of both cubes
    if pair != "mesh-box":
      sel = [k for k in range(n1) if p1[k][0] < 0.5]
      assert np.allclose(np.array(_as_sets(p1[sel])), np.array(_as_sets(p2[[k for k in range(n2) if p2[k][0] < 0.5]])), atol=1e-6)
    xpos = od_xpos(om, w)
    xmat = om.xmat[w].reshape(-1, 3, 3)
    for k in range(n1):
      bodies = (1, 2) if p1[k][0] < 0.5 else (3, 4)
      for b in bodies:
        loc = xmat[b].T @ (p1[k] - xpos[b])
        assert np.abs(loc).max() <= 0.1 + abs(d1[k]) + 1e-9, (w, k, b, loc)
  assert total >= 6 * 2 * 3  # multi-contact in every world on both pairs
  if pair == "mesh-box":
    return  # the multi-contact branch taken depends on which geom is geom1: only the same order compares
  # tilted past the face tolerance: the same (edge / single-contact) branch on both
  qpos = _states(mm, 4, seed=1, tilt=0.02)
  om, ob = _oracle(mm, qpos), _oracle(mb, qpos)
  for w in range(4):
    assert int(om.ncon[w, 0]) == int(ob.ncon[w, 0])


def od_xpos(od, w):
  return od.xpos[w].reshape(-1, 3)


def test_oracle_without_multiccd_one_contact_per_mesh_pair():
  mm = _load(MESH, MESH, flag="disable")
  od = _oracle(mm, _states(mm, 3))
  for w in range(3):
    n, _, _, _, geoms = _contacts(od, w)
    assert n == 2  # one per pair
  # box-box keeps its multi-contact whatever the flag (collision_convex.py:809)
  mb = _load(BOX, BOX, flag="disable")
  ob = _oracle(mb, _states(mb, 3))
  assert all(int(ob.ncon[w, 0]) > 2 for w in range(3))


def test_multiccd_margin_is_rejected():
  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf

  mjm = mjcf.load_model_from_string(SCENE.format(flag="enable", cube=CUBE, a=MESH + ' margin=".01"', b=MESH))
  with pytest.raises(NotImplementedError, match="MULTICCD"):
    mjw.put_model(mjm, device="cpu")


@pytest.mark.parametrize("pair", ["mesh-mesh", "box-mesh", "box-box"])
def test_oracle_turned_pair_quad_is_a_structural_tie(pair):
  """The turned pair's clipped polygon (the overlap of a square and the same square turned 25 degrees) has
  pairs of parallel edges, and _area4(a, b, c, d) is linear in d with no change along b - a: moving d along an
  edge parallel to a - b leaves the area unchanged in exact arithmetic.  _polygon_quad's first move compares
  two such areas (relative difference ~1e-7 from the 2e-4 tilt), so fp32 rounding decides it.  Pinned here:
  in most worlds the search meets such a near-tie, and the fp32 and FMA-contracted fp32 oracles each keep one
  of the quads the search reaches when every near-tie may go either way (reachable_quads on the fp64 polygon)."""
  a, b = {"mesh-mesh": (MESH, MESH), "box-mesh": (BOX, MESH), "box-box": (BOX, BOX)}[pair]
  mjm = _load(a, b)
  nworld = 16
  qpos = _states(mjm, nworld, seed=3)
  ods = {}
  for bits in (32, "32f"):
    _, od = oracle_from_state(mjm, qpos, np.zeros((nworld, mjm.nv)), np.zeros((nworld, mjm.nu)), njmax=128, nconmax=32, real_bits=bits)
    od.fwd_position()
    ods[bits] = od
  ties = 0
  for w in range(nworld):
    mine, cands, tie = turned_pair_candidates(mjm, qpos[w])
    ties += tie
    assert len(cands) <= 4
    assert any(same_points(mine, c, 1e-9) for c in cands)
    for bits, od in ods.items():
      _, _, p, _, _ = _contacts(od, w)
      assert any(same_points(p[p[:, 0] > 0.5], c) for c in cands), (w, bits)
  assert ties >= (2 if pair == "mesh-mesh" else nworld - 2), ties


@pytest.mark.gpu
@pytest.mark.parametrize("pair", ["mesh-mesh", "box-mesh", "box-box"])
def test_gpu_multiccd_matches_oracle(pair):
  import torch

  import mujoco_warp_amd as mjw

  a, b = {"mesh-mesh": (MESH, MESH), "box-mesh": (BOX, MESH), "box-box": (BOX, BOX)}[pair]
  mjm = _load(a, b)
  nworld = 16
  qpos = _states(mjm, nworld, seed=3)
  z = np.zeros((nworld, mjm.nv))
  m, d = gpu_from_state(mjm, qpos, z, np.zeros((nworld, mjm.nu)), njmax=128, nconmax=32)
  od = _oracle(mjm, qpos)
  _, o32f = oracle_from_state(mjm, qpos, z, np.zeros((nworld, mjm.nu)), njmax=128, nconmax=32, real_bits="32f")
  o32f.fwd_position()
  p32f = []
  for w in range(nworld):
    _, _, p, _, _ = _contacts(o32f, w)
    p32f.append(p[p[:, 0] > 0.5])
  hits32f = 0
  mjw.fwd_position(m, d)
  torch.cuda.synchronize()
  n = int(d.nacon[0])
  wid = np_(d.contact.worldid)[:n]
  for w in range(nworld):
    sel = np.nonzero(wid == w)[0]
    n2, d2, p2, f2, _ = _contacts(od, w)
    assert len(sel) == n2, (w, len(sel), n2)
    np.testing.assert_allclose(np.sort(np_(d.contact.dist)[sel]), np.sort(d2), atol=2e-5)
    gp = np_(d.contact.pos)[sel].astype(np.float64)
    # the first pair (a 4-corner overlap rectangle): the oracle's points, within fp32 rounding
    assert same_points(gp[gp[:, 0] < 0.5], p2[p2[:, 0] < 0.5]), w
    # the turned pair clips to a polygon of more than 4 vertices, of which polygon_quad keeps 4 by a greedy
    # search whose first move is a structural near-tie (test_oracle_turned_pair_quad_is_a_structural_tie):
    # every device point is a vertex of the oracle's clipped polygon (2e-4), and the 4 are a quad that search
    # keeps when its near-ties go either way
    _, cands, _ = turned_pair_candidates(mjm, qpos[w])
    gt = gp[gp[:, 0] > 0.5]
    assert any(same_points(gt, c) for c in cands), (w, gt, cands)
    hits32f += same_points(gt, p32f[w])
  print(f"{pair}: device turned-pair quad equals the FMA-contracted fp32 oracle's in {hits32f} of {nworld} worlds")


@pytest.mark.gpu
def test_gpu_mesh_mesh_ccd_kat_through_pipeline():
  """collision_gjk_test.py:470-488 test_mesh_mesh_ccd on the device: the two mesh cubes collide in 4 points."""
  import torch

  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf

  xml = f"""<mujoco><option><flag multiccd="enable"/></option><asset><mesh name="smallbox" vertex="{CUBE}"/></asset>
  <worldbody><geom pos="0 0 2" type="mesh" name="box1" mesh="smallbox"/>
  <body pos="0 1 3.99" euler="0 0 40"><freejoint/><geom type="mesh" name="box2" mesh="smallbox"/></body></worldbody></mujoco>"""
  mjm = mjcf.load_model_from_string(xml)
  m, d = gpu_from_state(mjm, mjm.qpos0[None], np.zeros((1, mjm.nv)), np.zeros((1, mjm.nu)), njmax=64, nconmax=8)
  mjw.fwd_position(m, d)
  torch.cuda.synchronize()
  assert int(d.nacon[0]) == 4
