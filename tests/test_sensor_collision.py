"""Collision sensors -- distance / normal / fromto (sensor.py:604-680, 710-757) -- and insidesite
(sensor.py:681-697, util_misc.py:603-632).

The reference's test_sensor_collision / test_sensor_collision_plane (sensor_test.py:680-830) compare against
MuJoCo C at run time and store no values, so the oracle is pinned here by analytic answers: two spheres'
surface distance, normal and nearest points; a body's distance is the minimum over its geoms; swapping
obj and ref flips the normal and the fromto segment; a cutoff of 0 reports 0 (and a zero normal / segment)
for separated geoms and clamps nothing for fromto; a box over a plane reports its lowest corner's height.
Convex pairs (collision_convex.py:763-852 with the sensor cutoff 1e32: GJK distance when separated, EPA depth
when overlapping, the frame flipped) are pinned by boxes: the gap between two aligned boxes and their facing
points, the overlap depth of two interpenetrating ones.  `-m gpu`: the sensor kernel against the oracle on the
reference's collision-sensor layouts (sensor_test.py:689-777), primitive and convex type sets, and on
overlapping box pairs."""

import numpy as np
import pytest

from tests.common import gpu_from_state, np_, oracle_from_state

SPHERES = """<mujoco><worldbody>
<body name="a"><geom name="a" type="sphere" size=".1"/></body>
<body name="b" pos="0.3 0.4 0"><freejoint/><geom name="b" type="sphere" size=".2"/>
  <geom name="b2" type="sphere" size=".05" pos="-.1 -.2 0"/></body>
<body name="c" pos="2 0 0"><geom name="c" type="box" size=".1 .2 .3"/><site name="zone" type="box" size=".5 .5 .5"/></body>
</worldbody>
<sensor>
  <distance geom1="a" geom2="b" cutoff="10"/>
  <distance geom1="b" geom2="a" cutoff="10"/>
  <normal geom1="a" geom2="b" cutoff="10"/>
  <normal geom1="b" geom2="a" cutoff="10"/>
  <fromto geom1="a" geom2="b" cutoff="10"/>
  <fromto geom1="b" geom2="a" cutoff="10"/>
  <distance geom1="a" body2="b" cutoff="10"/>
  <distance geom1="a" geom2="b" cutoff="0"/>
  <normal geom1="a" geom2="b" cutoff="0"/>
  <fromto geom1="a" geom2="b" cutoff="0"/>
  <insidesite site="zone" objtype="body" objname="c"/>
  <insidesite site="zone" objtype="body" objname="a"/>
</sensor></mujoco>"""


def _load(xml):
  from mujoco_warp_amd import mjcf

  return mjcf.load_model_from_string(xml)


def _oracle_sensors(mjm, qpos=None):
  qpos = mjm.qpos0[None] if qpos is None else qpos
  n = len(qpos)
  _, od = oracle_from_state(mjm, qpos, np.zeros((n, mjm.nv)), np.zeros((n, mjm.nu)))
  od.forward()
  return od.sensordata


def test_oracle_sphere_pair_known_answers():
  mjm = _load(SPHERES)
  sd = _oracle_sensors(mjm)[0]
  c = 0.5  # |(0.3, 0.4)|
  u = np.array([0.6, 0.8, 0.0])
  np.testing.assert_allclose(sd[0:2], [c - 0.3, c - 0.3], atol=1e-12)
  np.testing.assert_allclose(sd[2:5], u, atol=1e-12)
  np.testing.assert_allclose(sd[5:8], -u, atol=1e-12)
  np.testing.assert_allclose(sd[8:14], np.r_[0.1 * u, 0.3 * u], atol=1e-12)  # surface of a, then of b
  np.testing.assert_allclose(sd[14:20], np.r_[0.3 * u, 0.1 * u], atol=1e-12)
  # the body also holds b2 at (0.2, 0.2): |.| - 0.15 < 0.2
  np.testing.assert_allclose(sd[20], np.hypot(0.2, 0.2) - 0.15, atol=1e-12)
  # cutoff 0: separated geoms report the cutoff, a zero normal and a zero segment
  np.testing.assert_allclose(sd[21:31], 0.0, atol=0)
  np.testing.assert_array_equal(sd[31:33], [1.0, 0.0])


def test_oracle_plane_box_lowest_corner():
  mjm = _load("""<mujoco><worldbody><geom name="floor" type="plane" size="5 5 .1"/>
  <body name="b" pos="0 0 1" euler="10 20 30"><freejoint/><geom name="box" type="box" size=".1 .2 .3"/></body></worldbody>
  <sensor><distance geom1="floor" geom2="box" cutoff="10"/><fromto geom1="box" geom2="floor" cutoff="10"/></sensor></mujoco>""")
  _, od = oracle_from_state(mjm, mjm.qpos0[None], np.zeros((1, mjm.nv)), np.zeros((1, mjm.nu)))
  od.forward()
  R = od.geom_xmat[0].reshape(-1, 3, 3)[1]
  corners = np.array([[sx, sy, sz] for sx in (-.1, .1) for sy in (-.2, .2) for sz in (-.3, .3)]) @ R.T + od.geom_xpos[0].reshape(-1, 3)[1]
  low = corners[np.argmin(corners[:, 2])]
  sd = od.sensordata[0]
  np.testing.assert_allclose(sd[0], low[2], atol=1e-12)
  np.testing.assert_allclose(sd[1:4], low, atol=1e-12)  # from the box corner ...
  np.testing.assert_allclose(sd[4:7], [low[0], low[1], 0.0], atol=1e-12)  # ... to the plane


HFSENS = """<mujoco><asset><hfield name="h" nrow="3" ncol="4" size=".6 .5 .2 .1" elevation="0 0 0 0 0 0 0 0 0 0 0 0"/></asset>
<worldbody><geom name="hf" type="hfield" hfield="h" margin=".05"/>
<body name="s" pos=".1 .05 {z}"><freejoint/><geom name="s" type="{kind}" size=".1 .08 .06"/></body></worldbody>
<sensor><distance geom1="hf" geom2="s" cutoff="10"/><normal geom1="hf" geom2="s" cutoff="10"/>
<fromto geom1="s" geom2="hf" cutoff="10"/></sensor></mujoco>"""


@pytest.mark.parametrize("z", [0.09, 0.13, 0.5])
def test_oracle_hfield_sensor_sphere(z):
  """A sphere over a flat heightfield (collision_convex.py:158-697 for a sensor pair): the prism contacts'
  smallest distance while the pair passes the heightfield filter (within the 0.05 margin); beyond it the pair
  yields no contact and the sensor reports its cutoff.  The heightfield path reports distances of the
  margin-inflated shapes with no correction -- the prism top raised by the margin (:399, :425) and geom2
  inflated by half of it in support() -- so the distance is z - r - 1.5 margin."""
  import mujoco_warp_amd as mjw

  mjm = _load(HFSENS.format(z=z, kind="sphere"))
  assert mjw.put_model(mjm, device="cpu").nsensorccd == 3
  sd = _oracle_sensors(mjm)[0]
  if z < 0.2:
    np.testing.assert_allclose(sd[0], z - 0.1 - 0.075, atol=1e-6)
    np.testing.assert_allclose(np.abs(sd[3]), 1.0, atol=1e-6)
    np.testing.assert_allclose(np.linalg.norm(sd[7:10] - sd[4:7]), abs(z - 0.175), atol=1e-6)
  else:
    assert sd[0] == 10.0 and np.all(sd[1:] == 0)


BOXES = """<mujoco><worldbody><body name="a"><geom name="a" type="box" size=".1 .2 .3"/></body>
<body name="b" pos="0.02 -0.03 {z}"><freejoint/><geom name="b" type="box" size=".15 .1 .05"/></body></worldbody>
<sensor><distance geom1="a" geom2="b" cutoff="10"/><normal geom1="a" geom2="b" cutoff="10"/>
<fromto geom1="a" geom2="b" cutoff="10"/><distance geom1="b" geom2="a" cutoff="10"/><normal geom1="b" geom2="a" cutoff="10"/>
<distance geom1="a" geom2="b" cutoff="0"/></sensor></mujoco>"""


def test_put_model_accepts_convex_collision_sensors():
  import mujoco_warp_amd as mjw

  mjm = _load(BOXES.format(z=1))
  m = mjw.put_model(mjm, device="cpu")
  assert m.nsensorccd == 6 and m.nsensorcollision == 6
  assert m.ccd_epa_iterations == 16  # every convex pair (the sensors') is box-box (collision_convex.py:1127)


@pytest.mark.parametrize("z", [1.0, 0.33])
def test_oracle_convex_sensor_boxes(z):
  """Aligned boxes along z: separated by z - 0.35 (GJK distance), or overlapping by 0.35 - z (EPA depth); the
  normal from a to b is +z, the fromto ends lie on the facing faces (the overlap's points on b's bottom / a's
  top face), and swapping the geoms negates the normal."""
  mjm = _load(BOXES.format(z=z))
  sd = _oracle_sensors(mjm)[0]
  gap = z - 0.35
  np.testing.assert_allclose(sd[0], gap, atol=1e-6)
  np.testing.assert_allclose(sd[1:4], [0, 0, 1], atol=1e-6)
  np.testing.assert_allclose([sd[6], sd[9]], [0.3, z - 0.05] if gap > 0 else [z - 0.05, 0.3], atol=1e-6)
  np.testing.assert_allclose(np.linalg.norm(sd[7:10] - sd[4:7]), abs(gap), atol=1e-6)
  np.testing.assert_allclose(sd[10], gap, atol=1e-6)
  np.testing.assert_allclose(sd[11:14], [0, 0, -1], atol=1e-6)
  np.testing.assert_allclose(sd[14], 0.0 if gap > 0 else gap, atol=1e-6)  # cutoff 0 clamps positive distances


# the reference's collision-sensor layout (sensor_test.py:689-777) over primitive pairs
LAYOUT = """<mujoco><worldbody>
  <body name="obj0"><freejoint/><geom name="obj0" type="{0}" size=".1 .1 .1" euler="1 2 3"/></body>
  <body name="obj1" pos="0 0 1"><freejoint/><geom name="obj1" type="{1}" size=".1 .1 .1" euler="-1 2 -1"/></body>
  <body name="objobj" pos="0 0 -1"><freejoint/>
    <geom name="objobj0" pos=".01 0 0.005" type="{2}" size=".09 .09 .09" euler="2 1 3"/>
    <geom name="objobj1" pos="-.01 0 -0.0025" type="{3}" size=".11 .11 .11" euler="3 1 2"/>
  </body>
  <body name="probe" pos=".05 0 .95"><freejoint/><geom type="sphere" size=".01" contype="0" conaffinity="0"/></body>
  <site name="zone" pos="0 0 1" type="{1}" size=".1 .1 .1" euler="-1 2 -1"/>
</worldbody>
<sensor>
{sensors}
  <insidesite site="zone" objtype="body" objname="probe"/>
  <insidesite site="zone" objtype="xbody" objname="obj0"/>
</sensor></mujoco>"""


def _layout(types_):
  rows = []
  for kind in ("distance", "normal", "fromto"):
    for a, b in (("geom1=\"obj0\"", "geom2=\"obj1\""), ("geom1=\"obj1\"", "geom2=\"obj0\""), ("body1=\"obj0\"", "body2=\"obj1\""),
                 ("geom1=\"obj0\"", "body2=\"objobj\""), ("body1=\"objobj\"", "geom2=\"obj0\""), ("body1=\"obj0\"", "body2=\"objobj\"")):
      for cutoff in ("0", "10"):
        rows.append(f"  <{kind} {a} {b} cutoff=\"{cutoff}\"/>")
  return _load(LAYOUT.format(*types_, sensors="\n".join(rows)))


PRIMITIVE_SETS = [("sphere", "capsule", "capsule", "sphere"), ("capsule", "sphere", "box", "capsule"), ("sphere", "sphere", "box", "cylinder"),
                  ("capsule", "capsule", "sphere", "box")]
# sets with convex (GJK) pairs: box-box, ellipsoid / cylinder against the rest
CONVEX_SETS = [("box", "box", "box", "box"), ("ellipsoid", "cylinder", "box", "sphere"), ("cylinder", "box", "capsule", "ellipsoid"),
               ("box", "ellipsoid", "cylinder", "cylinder")]


def test_oracle_layout_invariants():
  """Swapping obj and ref negates the normal and swaps the fromto ends; fromto length = distance."""
  mjm = _layout(PRIMITIVE_SETS[0])
  sd = _oracle_sensors(mjm)[0]
  n = 12  # per kind: 6 obj/ref combos x 2 cutoffs
  dist, nrm, ft = sd[:n], sd[n:n + 3 * n].reshape(n, 3), sd[4 * n:4 * n + 6 * n].reshape(n, 6)
  np.testing.assert_allclose(dist[1], dist[3])  # geom-geom both ways, cutoff 10
  np.testing.assert_allclose(nrm[1], -nrm[3], atol=1e-12)
  np.testing.assert_allclose(ft[1], np.r_[ft[3][3:], ft[3][:3]], atol=1e-12)
  np.testing.assert_allclose(np.linalg.norm(ft[1][3:] - ft[1][:3]), abs(dist[1]), atol=1e-9)
  assert dist[0] == 0.0 and np.all(nrm[0] == 0) and np.all(ft[0] == 0)  # cutoff 0, separated


def test_oracle_convex_layout_invariants():
  """The layout's invariants hold on the convex path too (GJK witness points, flipped frame)."""
  mjm = _layout(CONVEX_SETS[1])
  sd = _oracle_sensors(mjm)[0]
  n = 12
  dist, nrm, ft = sd[:n], sd[n:n + 3 * n].reshape(n, 3), sd[4 * n:4 * n + 6 * n].reshape(n, 6)
  np.testing.assert_allclose(dist[1], dist[3], atol=1e-9)
  np.testing.assert_allclose(nrm[1], -nrm[3], atol=1e-6)
  np.testing.assert_allclose(np.linalg.norm(ft[1][3:] - ft[1][:3]), abs(dist[1]), atol=1e-6)
  np.testing.assert_allclose((ft[1][3:] - ft[1][:3]) / dist[1], nrm[1], atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("types_", PRIMITIVE_SETS + CONVEX_SETS)
def test_gpu_collision_sensors_match_oracle(types_):
  import torch

  import mujoco_warp_amd as mjw

  mjm = _layout(types_)
  nworld = 8
  rng = np.random.default_rng(11)
  qpos = np.tile(mjm.qpos0, (nworld, 1))
  for j in range(mjm.njnt):  # free joints: move and turn every body a little per world
    a = mjm.jnt_qposadr[j]
    qpos[1:, a:a + 3] += rng.normal(0, 0.05, (nworld - 1, 3))
    q = qpos[1:, a + 3:a + 7] + rng.normal(0, 0.2, (nworld - 1, 4))
    qpos[1:, a + 3:a + 7] = q / np.linalg.norm(q, axis=1, keepdims=True)
  qvel = np.zeros((nworld, mjm.nv))
  ctrl = np.zeros((nworld, mjm.nu))
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl)
  mjw.forward(m, d)
  od.forward()
  torch.cuda.synchronize()
  got, want = np_(d.sensordata), od.sensordata
  if types_ in PRIMITIVE_SETS:
    np.testing.assert_allclose(got, want, rtol=1e-5, atol=2e-6)
  else:
    # GJK distance of separated convex geoms: the distance converges to the ccd tolerance (1e-6); the witness
    # points of smooth supports (ellipsoid, cylinder) to its square root
    n = 12
    np.testing.assert_allclose(got[:, :n], want[:, :n], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(got[:, n:], want[:, n:], atol=2e-3)
  assert np.abs(want[:, 1:12:2]).max() > 0.05  # cutoff-10 distances are real distances


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["sphere", "box", "capsule"])
def test_gpu_hfield_sensors_match_oracle(kind):
  import torch

  import mujoco_warp_amd as mjw

  mjm = _load(HFSENS.format(z=0.1, kind=kind))
  nworld = 6
  rng = np.random.default_rng(8)
  qpos = np.tile(mjm.qpos0, (nworld, 1))
  qpos[:, 2] = rng.uniform(0.02, 0.16, nworld)
  q = qpos[:, 3:7] + rng.normal(0, 0.3, (nworld, 4))
  qpos[:, 3:7] = q / np.linalg.norm(q, axis=1, keepdims=True)
  m, d = gpu_from_state(mjm, qpos, np.zeros((nworld, mjm.nv)), np.zeros((nworld, mjm.nu)))
  _, od = oracle_from_state(mjm, qpos, np.zeros((nworld, mjm.nv)), np.zeros((nworld, mjm.nu)))
  mjw.forward(m, d)
  od.forward()
  torch.cuda.synchronize()
  got, want = np_(d.sensordata), od.sensordata
  np.testing.assert_allclose(got[:, 0], want[:, 0], atol=5e-5)  # the smallest prism-contact distance
  seg = got[:, 7:10] - got[:, 4:7]
  np.testing.assert_allclose(np.linalg.norm(seg, axis=1), np.minimum(np.abs(got[:, 0]), 10.0) * (got[:, 0] < 10), atol=5e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("z", [1.0, 0.33, 0.3])
def test_gpu_convex_sensor_boxes(z):
  """BOXES on the device (GJK when separated, EPA + box multi-contact's first point when overlapping),
  turned a little per world, against the oracle."""
  import torch

  import mujoco_warp_amd as mjw

  mjm = _load(BOXES.format(z=z))
  nworld = 6
  rng = np.random.default_rng(4)
  qpos = np.tile(mjm.qpos0, (nworld, 1))
  q = qpos[1:, 3:7] + rng.normal(0, 0.05, (nworld - 1, 4))
  qpos[1:, 3:7] = q / np.linalg.norm(q, axis=1, keepdims=True)
  m, d = gpu_from_state(mjm, qpos, np.zeros((nworld, mjm.nv)), np.zeros((nworld, mjm.nu)))
  _, od = oracle_from_state(mjm, qpos, np.zeros((nworld, mjm.nv)), np.zeros((nworld, mjm.nu)))
  mjw.forward(m, d)
  od.forward()
  torch.cuda.synchronize()
  got, want = np_(d.sensordata), od.sensordata
  np.testing.assert_allclose(got[:, [0, 10, 14]], want[:, [0, 10, 14]], atol=2e-5)
  cols = [c for c in range(got.shape[1]) if not 4 <= c < 10]
  np.testing.assert_allclose(got[:, cols], want[:, cols], atol=5e-4)
  # fromto against the fp32 oracle (liborc32) at 5e-4.  Overlapping boxes give several multi-contact points at
  # one depth, and the sensor reports the first: where the clipped polygon's start is a rounding tie (two
  # coplanar EPA faces, duplicate points of an edge-face clip), the fp32 oracle compiled with the device's
  # fused multiply-adds (liborc32f) can pick another point than the sequential builds -- at z = 0.33, world 2,
  # it picks the device's.  In a world with several equal-depth contacts whose builds disagree, the device's
  # segment must be one of the oracle's contact points' segments (pos -+ dist / 2 along the normal).
  _, o32 = oracle_from_state(mjm, qpos, np.zeros((nworld, mjm.nv)), np.zeros((nworld, mjm.nu)), real_bits=32)
  _, o32f = oracle_from_state(mjm, qpos, np.zeros((nworld, mjm.nv)), np.zeros((nworld, mjm.nu)), real_bits="32f")
  o32.forward()
  o32f.forward()
  w32, w32f = np.asarray(o32.sensordata, np.float64), np.asarray(o32f.sensordata, np.float64)
  ties = 0
  for w in range(nworld):
    n = int(od.ncon[w, 0])
    if n <= 1 or np.abs(w32[w, 4:10] - w32f[w, 4:10]).max() < 5e-4 and np.abs(got[w, 4:10] - w32[w, 4:10]).max() < 5e-4:
      # one contact (no order to tie), or every build agrees: the strict comparison
      np.testing.assert_allclose(got[w, 4:10], w32[w, 4:10], atol=5e-4, err_msg=f"world {w}")
      continue
    ties += 1
    segs = []
    for c in range(n):
      p, dd, nn = od.con_pos[w, 3 * c:3 * c + 3], od.con_dist[w, c], od.con_frame[w, 9 * c:9 * c + 3]
      segs.append(np.sort(np.stack([p - 0.5 * dd * nn, p + 0.5 * dd * nn]), axis=0))
    mine = np.sort(np.stack([got[w, 4:7], got[w, 7:10]]).astype(np.float64), axis=0)
    assert min(np.abs(s_ - mine).max() for s_ in segs) < 5e-4, (w, got[w, 4:10], segs)
  assert ties <= 2  # world 2 at z = 0.33 and 0.3 (four contacts at one depth, two of them duplicated)


@pytest.mark.gpu
@pytest.mark.parametrize("geom", ["sphere", "capsule", "ellipsoid", "cylinder", "box"])
def test_gpu_collision_sensors_plane(geom):
  """sensor_test.py:787-830's plane layout (plane against each primitive), device against the oracle."""
  import torch

  import mujoco_warp_amd as mjw

  mjm = _load(f"""<mujoco><worldbody><geom name="plane" type="plane" size="10 10 .01"/>
  <body name="b" pos="0 0 .5" euler="10 20 30"><freejoint/><geom name="g" type="{geom}" size=".1 .15 .2"/></body></worldbody>
  <sensor><distance geom1="plane" geom2="g" cutoff="10"/><distance geom1="g" geom2="plane" cutoff="10"/>
  <normal geom1="plane" geom2="g" cutoff="10"/><normal geom1="g" geom2="plane" cutoff="10"/>
  <fromto geom1="plane" geom2="g" cutoff="10"/><fromto geom1="g" geom2="plane" cutoff="10"/></sensor></mujoco>""")
  nworld = 4
  rng = np.random.default_rng(3)
  qpos = np.tile(mjm.qpos0, (nworld, 1))
  q = qpos[:, 3:7] + rng.normal(0, 0.3, (nworld, 4))
  qpos[:, 3:7] = q / np.linalg.norm(q, axis=1, keepdims=True)
  qpos[:, 2] = rng.uniform(0.05, 0.6, nworld)
  m, d = gpu_from_state(mjm, qpos, np.zeros((nworld, mjm.nv)), np.zeros((nworld, mjm.nu)))
  om, od = oracle_from_state(mjm, qpos, np.zeros((nworld, mjm.nv)), np.zeros((nworld, mjm.nu)))
  mjw.forward(m, d)
  od.forward()
  torch.cuda.synchronize()
  np.testing.assert_allclose(np_(d.sensordata), od.sensordata, rtol=1e-5, atol=2e-6)
