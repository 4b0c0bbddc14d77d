"""tactile sensor (sensor.py:2085-2252 _preprocess_tactile_contacts / _sensor_tactile; MuJoCo's mjSENS_TACTILE).

One taxel per vertex of the sensor's mesh, placed with the sensor geom's pose; each taxel takes pressure
depth / max(0.05 - depth, MINVAL) from every distinct contact partner of the sensor geom's weld body whose
primitive SDF (collision_sdf.py:157-183, 393-400) is negative there.  The output is [normal (nvt), slip 1
(nvt), slip 2 (nvt)]; the slip terms need per-vertex tangent frames, which this compiler's meshes do not
carry, so they are 0 (as in the reference for such meshes, sensor.py:2181-2190, 2245-2247).

Parity: MuJoCo is not importable here, and the reference's own tactile tests (sensor_test.py:895-937,
io_test.py collision_sdf/tactile.xml) compare against MuJoCo C on builtin meshes and an SDF plugin this
compiler does not generate, so the oracle is pinned by known answers computed in numpy from the scene's
geometry: a pad pressed into a plane (uniform depth; four floor contacts deduplicated to one partner), a
tilted pad (per-taxel depth from the rotation), a pad on a box (the radial-field interior SDF), a pad on a
sphere (only the taxels inside it) and a lifted pad (no contacts: zeros).  Under `-m gpu` the device sensor
kernel follows the oracle on the same worlds.
"""

import numpy as np
import pytest

from tests.common import gpu_from_state, np_, oracle_from_state

_G = [-.08, 0.0, .08]
# the pad: a 3 x 3 grid of taxels on its flat face and an apex 1 cm above it (a closed low pyramid)
_VERTS = [(x, y, 0.0) for y in _G for x in _G] + [(0.0, 0.0, 0.01)]
_FACES = []
for j in range(2):
  for i in range(2):
    a, b, c, d = 3 * j + i, 3 * j + i + 1, 3 * (j + 1) + i, 3 * (j + 1) + i + 1
    _FACES += [(a, c, b), (b, c, d)]
_RIM = [0, 1, 2, 5, 8, 7, 6, 3]
_FACES += [(_RIM[k], _RIM[(k + 1) % 8], 9) for k in range(8)]

XML = f"""<mujoco><option timestep="0.002"/>
<asset><mesh name="pad" vertex="{' '.join(f'{v:g}' for p in _VERTS for v in p)}" face="{' '.join(str(i) for f in _FACES for i in f)}"/></asset>
<worldbody>
  <geom name="floor" type="plane" size="5 5 .1"/>
  <geom name="table" type="box" pos="1 0 .1" size=".3 .3 .1"/>
  <geom name="dome" type="sphere" pos="-1 0 0" size=".2"/>
  <body name="finger" pos="0 0 .5"><freejoint/>
    <geom name="fbox" type="box" size=".1 .1 .1" mass="1"/>
    <geom name="fpad" type="mesh" mesh="pad" pos="0 0 -.11" contype="0" conaffinity="0" mass="0"/>
  </body>
</worldbody>
<sensor><tactile name="touchpad" geom="fpad" mesh="pad"/></sensor></mujoco>"""

_PAD_OFFSET = np.array([0.0, 0.0, -0.11])


def _load():
  from mujoco_warp_amd import mjcf

  return mjcf.load_model_from_string(XML)


def _quat_x(angle):
  return np.array([np.cos(angle / 2), np.sin(angle / 2), 0.0, 0.0])


def _rot(q):
  w, x, y, z = q
  return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                   [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                   [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


# the finger's free-joint poses of the five worlds: pressed into the floor, tilted on the floor, on the
# table box, on the dome sphere, lifted clear
POSES = [
  (np.array([0.0, 0.0, 0.095]), np.array([1.0, 0.0, 0.0, 0.0])),
  (np.array([0.0, 0.0, 0.099]), _quat_x(0.08)),
  (np.array([1.0, 0.0, 0.295]), np.array([1.0, 0.0, 0.0, 0.0])),
  (np.array([-1.0, 0.0, 0.295]), np.array([1.0, 0.0, 0.0, 0.0])),
  (np.array([0.0, 0.0, 0.5]), np.array([1.0, 0.0, 0.0, 0.0])),
]


def _qpos():
  return np.stack([np.concatenate([p, q]) for p, q in POSES])


def _pressure(depth):
  depth = np.minimum(depth, 0.0)
  return np.where(depth < 0, depth / np.maximum(0.05 - depth, 1e-15), 0.0)


def _box_sdf(p, size):
  """collision_sdf.py:163-171, restated independently of the C oracle."""
  a = np.abs(p) - size
  if np.any(a >= 0):
    return np.linalg.norm(np.maximum(a, 0)) + min(a.max(), 0.0)
  f = -size / a
  f = f / np.linalg.norm(f)
  return -np.min(-a / np.abs(f))


def _expected(world):
  pos, quat = POSES[world]
  taxels = pos + (_rot(quat) @ (np.array(_VERTS) + _PAD_OFFSET).T).T
  nvt = len(_VERTS)
  out = np.zeros(3 * nvt)
  if world in (0, 1):  # the floor plane: depth = z (one partner although the box has 4 floor contacts)
    out[:nvt] = _pressure(taxels[:, 2])
  elif world == 2:  # the table box
    out[:nvt] = [_pressure(_box_sdf(t - np.array([1.0, 0.0, 0.1]), np.array([.3, .3, .1]))) for t in taxels]
  elif world == 3:  # the dome sphere
    out[:nvt] = _pressure(np.linalg.norm(taxels - np.array([-1.0, 0.0, 0.0]), axis=1) - 0.2)
  return out


def _oracle(bits=64):
  mjm = _load()
  qpos = _qpos()
  n = len(POSES)
  _, od = oracle_from_state(mjm, qpos, np.zeros((n, mjm.nv)), np.zeros((n, mjm.nu)), njmax=128, nconmax=32, real_bits=bits)
  od.forward()
  return mjm, od


def test_compiler_tactile_layout():
  mjm = _load()
  s = mjm.sensor_names.index("touchpad")
  nvt = len(_VERTS)
  assert int(mjm.sensor_type[s]) == 46 and int(mjm.sensor_dim[s]) == 3 * nvt
  assert int(mjm.sensor_objtype[s]) == 10 and int(mjm.sensor_reftype[s]) == 5  # mesh, geom
  assert int(mjm.sensor_refid[s]) == mjm.geom_names.index("fpad")
  assert int(mjm.sensor_needstage[s]) == 3  # acceleration stage (after the contacts' constraint rows)
  # io.py:556-567: one taxel per mesh vertex
  from mujoco_warp_amd import io

  m = io.put_model(mjm)
  assert int(m.nsensortaxel) == nvt
  np.testing.assert_array_equal(np_(m.taxel_vertadr), np.arange(nvt))
  np.testing.assert_array_equal(np_(m.taxel_sensorid), np.zeros(nvt))
  # unit vertex normals; the grid's interior taxel faces straight down
  nrm = np.asarray(mjm.mesh_normal).reshape(-1, 3)
  np.testing.assert_allclose(np.linalg.norm(nrm, axis=1), 1.0, atol=1e-12)
  np.testing.assert_allclose(nrm[4], [0.0, 0.0, -1.0], atol=1e-12)


def test_oracle_tactile_known_answers():
  mjm, od = _oracle()
  a = int(mjm.sensor_adr[0])
  nvt = len(_VERTS)
  gid = {n: i for i, n in enumerate(mjm.geom_names)}
  for w in range(len(POSES)):
    ncon = int(od.ncon[w, 0]) if od.ncon.ndim == 2 else int(od.ncon[w])
    geoms = od.con_geom[w].reshape(-1, 2)[:ncon]
    if w == 0:
      assert sum(gid["floor"] in g for g in geoms) == 4  # four floor contacts, one partner
    if w == 4:
      assert ncon == 0
    got = od.sensordata[w][a:a + 3 * nvt]
    want = _expected(w)
    np.testing.assert_allclose(got, want, rtol=1e-9, atol=1e-12, err_msg=f"world {w}")
  # every pose but the lifted one presses something
  for w in range(4):
    assert np.all(od.sensordata[w][a:a + nvt] <= 0) and od.sensordata[w][a:a + nvt].min() < -0.1
  # the dome: only the taxels inside the sphere (the grid's centre and the apex)
  assert np.flatnonzero(od.sensordata[3][a:a + nvt]).tolist() == [4, 9]


def test_oracle_tactile_fp32_tracks_fp64():
  _, a = _oracle(64)
  _, b = _oracle(32)
  np.testing.assert_allclose(np.asarray(b.sensordata, np.float64), a.sensordata, rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("sparse", [False, True], ids=["dense", "sparse"])
def test_gpu_tactile_matches_oracle(sparse):
  """The sensor kernel serves both pipelines: the dense world-per-wave one and (jacobian = sparse) the
  workgroup-per-world sparse one, whose contacts reach it through the same constraint rows."""
  import torch

  import mujoco_warp_amd as mjw

  mjm, od = _oracle()
  if sparse:
    mjm = _load()
    mjm.opt.jacobian = 1
  qpos = _qpos()
  n = len(POSES)
  m, d = gpu_from_state(mjm, qpos, np.zeros((n, mjm.nv)), np.zeros((n, mjm.nu)), njmax=128, nconmax=32)
  mjw.forward(m, d)
  torch.cuda.synchronize()
  a, nvt = int(mjm.sensor_adr[0]), len(_VERTS)
  got = np_(d.sensordata)[:, a:a + 3 * nvt]
  want = od.sensordata[:, a:a + 3 * nvt]
  # fp32 device geometry vs the fp64 oracle: depths of ~1e-2 to ~1e-6 relative
  np.testing.assert_allclose(got, want, rtol=1e-4, atol=2e-5)
  for w in range(n):
    np.testing.assert_allclose(got[w], _expected(w), rtol=1e-4, atol=2e-5, err_msg=f"world {w}")
