"""contact sensor (sensor.py:1750-1940 output, 2258-2430 matching and reduction; MuJoCo's mjSENS_CONTACT).

Matches are taken in the world's contact order (MuJoCo C's order; the reference's atomic match order is
arbitrary, and its mindist / maxforce sort restores a criteria order, which is what is compared), at most
Option.contact_sensor_maxmatch of them.  The oracle is pinned by known answers on resting bodies: the
found count equals the number of contacts on the named object, netforce carries the weight of the
supported bodies, mindist reports the deepest contact, matching by subtree covers a body's children, a site
zone keeps only the contacts inside it, and obj / ref order flips the normal.  Under `-m gpu` the device
sensor kernel follows the oracle on the same contacts (contact set and forces from the same solver state).
"""

import numpy as np
import pytest

from tests.common import gpu_from_state, np_, oracle_from_state

XML = """<mujoco><option timestep="0.002"/>
<worldbody>
  <geom name="floor" type="plane" size="5 5 .1"/>
  <body name="box" pos="0 0 .1"><freejoint/><geom name="boxg" type="box" size=".1 .1 .1" mass="2"/>
    <site name="corner" pos=".1 .1 -.1" size=".03"/>
  </body>
  <body name="ball" pos=".6 0 .1"><freejoint/><geom name="ballg" type="sphere" size=".1" mass="1"/></body>
  <body name="stack" pos="-.6 0 .1"><freejoint/><geom name="stack0" type="box" size=".1 .1 .1" mass="1"/>
    <body name="child" pos="0 0 .2"><joint type="slide" axis="0 0 1"/><geom name="stack1" type="sphere" size=".05" mass=".5"/></body>
  </body>
</worldbody>
<sensor>
  <contact name="box_found" body1="box" data="found"/>
  <contact name="box_net" body1="box" data="found force torque pos" reduce="netforce"/>
  <contact name="floor_box_mind" geom1="floor" geom2="boxg" num="2" data="found dist normal" reduce="mindist"/>
  <contact name="box_floor_mind" geom1="boxg" geom2="floor" num="2" data="found dist normal" reduce="mindist"/>
  <contact name="ball_none" geom1="ballg" num="3" data="found force pos normal tangent"/>
  <contact name="sub" subtree1="stack" num="4" data="found force" reduce="maxforce"/>
  <contact name="site" site="corner" num="2" data="found pos"/>
  <contact name="all" num="12" data="found dist"/>
</sensor></mujoco>"""


def _load():
  from mujoco_warp_amd import mjcf

  return mjcf.load_model_from_string(XML)


def _adr(mjm, name):
  s = mjm.sensor_names.index(name)
  return int(mjm.sensor_adr[s]), int(mjm.sensor_dim[s])


def _settled(mjm, nstep=300, bits=64):
  qpos = mjm.qpos0[None].copy()
  _, od = oracle_from_state(mjm, qpos, np.zeros((1, mjm.nv)), np.zeros((1, mjm.nu)), njmax=128, nconmax=32, real_bits=bits)
  for _ in range(nstep):
    od.step()
  od.forward()
  return od


def test_compiler_contact_sensor_layout():
  mjm = _load()
  s = mjm.sensor_names.index("box_net")
  assert int(mjm.sensor_intprm[s][0]) == 1 | 2 | 4 | 16 and int(mjm.sensor_intprm[s][1]) == 3
  assert int(mjm.sensor_dim[s]) == 1 + 3 + 3 + 3
  assert int(mjm.sensor_dim[mjm.sensor_names.index("ball_none")]) == 3 * (1 + 3 + 3 + 3 + 3)
  assert int(mjm.sensor_needstage[s]) == 3  # acceleration stage (efc_force)
  from mujoco_warp_amd import mjcf

  with pytest.raises(ValueError):
    mjcf.load_model_from_string(XML.replace('data="found dist normal" reduce="mindist"/>\n  <contact name="box_floor_mind"',
                                            'data="dist found" reduce="mindist"/>\n  <contact name="box_floor_mind"'))


def test_oracle_contact_sensor_known_answers():
  mjm = _load()
  od = _settled(mjm)
  sd = od.sensordata[0]
  ncon = int(od.ncon[0, 0])
  geoms = od.con_geom[0].reshape(-1, 2)[:ncon]
  gid = {n: i for i, n in enumerate(mjm.geom_names)}
  on_box = sum(gid["boxg"] in g for g in geoms)
  assert on_box == 4  # a resting box: four corners
  a, _ = _adr(mjm, "box_found")
  assert sd[a] == on_box
  # netforce: the four corner forces carry the box's weight (2 kg); centroid under the box centre
  a, _ = _adr(mjm, "box_net")
  assert sd[a] == 4
  g = 9.81 * 2.0
  np.testing.assert_allclose(abs(sd[a + 3]), g, rtol=2e-3)
  np.testing.assert_allclose(sd[a + 1:a + 3], 0.0, atol=1e-3 * g)
  box_xy = od.xpos[0].reshape(-1, 3)[mjm.body_names.index("box"), :2]
  np.testing.assert_allclose(sd[a + 7:a + 9], box_xy, atol=1e-3)
  # mindist: the deepest contact first, its normal flipped by obj / ref order
  a1, _ = _adr(mjm, "floor_box_mind")
  a2, _ = _adr(mjm, "box_floor_mind")
  dists = [od.con_dist[0][c] for c in range(ncon) if gid["boxg"] in geoms[c]]
  np.testing.assert_allclose(sd[a1 + 1], min(dists), rtol=0, atol=1e-15)
  assert sd[a1 + 1] <= sd[a1 + 5 + 1]  # slot order: ascending distance
  np.testing.assert_allclose(sd[a1 + 2:a1 + 5], -sd[a2 + 2:a2 + 5], atol=1e-15)
  # subtree: the stack's base box (4 floor corners) and its child sphere resting on it
  a, _ = _adr(mjm, "sub")
  assert sd[a] == sum((gid["stack0"] in gg) or (gid["stack1"] in gg) for gg in geoms) >= 5
  fz = [abs(sd[a + 4 * i + 1]) for i in range(4)]
  assert fz == sorted(fz, reverse=True)  # maxforce: the largest normal force first
  # site zone: only the corner contact under the site
  a, _ = _adr(mjm, "site")
  assert sd[a] == 1
  np.testing.assert_allclose(sd[a + 1:a + 3], [0.1, 0.1], atol=2e-3)
  assert np.all(sd[a + 4:a + 8] == 0)  # unused slot zeroed
  # no objects: every contact, in contact order
  a, dim = _adr(mjm, "all")
  assert sd[a] == ncon
  np.testing.assert_allclose(sd[a + 1:a + 2 * ncon:2], od.con_dist[0][:ncon], atol=0)


def test_oracle_contact_sensor_fp32_tracks_fp64():
  mjm = _load()
  a = _settled(mjm, 100, 64).sensordata[0]
  b = np.asarray(_settled(mjm, 100, 32).sensordata[0], np.float64)
  np.testing.assert_allclose(b, a, rtol=2e-3, atol=2e-3 * np.abs(a).max())


def test_oracle_contact_sensor_counts_contacts_without_rows():
  """sensor.py:2313-2316 keeps every CONSTRAINT contact, with rows or not: with njmax too small for the
  contact rows (4 box corners x 4 pyramid rows + the other bodies' contacts > 10), the found counts do not
  change, and a contact whose rows were cut reports zero force."""
  mjm = _load()
  od0 = _settled(mjm)
  qpos, warm = od0.qpos[:1].copy(), od0.qacc[:1].copy()
  _, od = oracle_from_state(mjm, qpos, np.zeros((1, mjm.nv)), np.zeros((1, mjm.nu)), njmax=10, nconmax=32, qacc_warmstart=warm)
  od.forward()
  assert int(od.nefc[0, 0]) > 10  # rows were requested past njmax and dropped
  ncon = int(od.ncon[0, 0])
  adr0 = od.con_efc_address[0].reshape(-1, 10)[:ncon, 0]
  assert (adr0 < 0).any()
  sd, sd0 = od.sensordata[0], od0.sensordata[0]
  for name in ("box_found", "all"):
    a, _ = _adr(mjm, name)
    assert sd[a] == sd0[a] == (4 if name == "box_found" else ncon)
  a, dim = _adr(mjm, "sub")
  assert sd[a] == sd0[a]


@pytest.mark.gpu
@pytest.mark.parametrize("njmax", [128, 10])
def test_gpu_contact_sensor_matches_oracle(njmax):
  import torch

  import mujoco_warp_amd as mjw

  mjm = _load()
  od0 = _settled(mjm, 200)
  nworld = 4
  rng = np.random.default_rng(1)
  qpos = np.tile(od0.qpos[0], (nworld, 1))
  qpos[1:, :3] += rng.normal(0, 0.003, (nworld - 1, 3))
  qvel = np.zeros((nworld, mjm.nv))
  ctrl = np.zeros((nworld, mjm.nu))
  warm = np.tile(od0.qacc[0], (nworld, 1))
  # njmax 10: the rows of most contacts are dropped, the contacts stay in the pool (found counts them)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=njmax, nconmax=32, qacc_warmstart=warm)
  _, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=njmax, nconmax=32, qacc_warmstart=warm)
  mjw.forward(m, d)
  od.forward()
  torch.cuda.synchronize()
  got, want = np_(d.sensordata), od.sensordata
  # counts and contact geometry exactly as the oracle's (same contacts, same order); forces carry the
  # iterative solve (the solver bar, tests/test_gpu_parity_models.py: qacc 5e-3 normwise)
  for w in range(nworld):
    for name in mjm.sensor_names:
      a, dim = _adr(mjm, name)
      np.testing.assert_allclose(got[w, a:a + dim], want[w, a:a + dim], rtol=5e-3, atol=5e-3 * max(1.0, np.abs(want[w, a:a + dim]).max()),
                                 err_msg=f"world {w} sensor {name}")
