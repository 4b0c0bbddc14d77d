"""Explicit <contact><pair> entries against the reference's own known-answer tests.

Vectors: tests/golden/pair_kat.json, extracted as data by tests/golden/make_golden_pair.py from
collision_driver_test.py::test_contact_pair (the nxn_pairid layout, nacon and the pair's contact
parameters: includemargin = margin - gap, dim, friction, solref, solreffriction, solimp) and
io_test.py::test_margin_pair_box_box (a box-box pair with a margin is refused).  The pair's parameters
replace the geom mix in contact_params (collision_core.py:270-277).  The oracle runs on the CPU, the HIP
forward kernel under -m gpu; a one-step rollout of a pair scene compares the two.
"""

import json
import os

import numpy as np
import pytest

from mujoco_warp_amd import mjcf
from mujoco_warp_amd.io import nxn_geom_pairs

KAT = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "pair_kat.json")))
CASES = KAT["contact_pair"]
IDS = [f"case{i}" for i in range(len(CASES))]


def _check_pairid(case, mjm):
  _, pid = nxn_geom_pairs(mjm, unfiltered=True)
  if "pairid_all" in case:
    assert (pid[:, 0] == case["pairid_all"]).all()
  if "pairid" in case:
    np.testing.assert_array_equal(pid[:, 0], case["pairid"])


def _check_contact(case, get):
  if "nacon" in case:
    assert get("nacon") == case["nacon"]
  i = case.get("contact_index", 0)
  for f, want in case["contact"].items():
    got = get(f)[i]
    np.testing.assert_allclose(got, want, rtol=1e-6, atol=1e-6, err_msg=f)


@pytest.mark.parametrize("case", CASES, ids=IDS)
def test_oracle_contact_pair_kat(case):
  from oracle import orc

  mjm = mjcf.load_model_from_string(case["xml"])
  _check_pairid(case, mjm)
  om = orc.OracleModel(mjm)
  od = orc.OracleData(om, 1, 64, 16)
  od.fwd_position()
  names = {"nacon": "ncon", "includemargin": "con_includemargin", "dim": "con_dim", "friction": "con_friction",
           "solref": "con_solref", "solreffriction": "con_solreffriction", "solimp": "con_solimp"}
  shapes = {"friction": 5, "solref": 2, "solreffriction": 2, "solimp": 5}

  def get(f):
    a = np.asarray(getattr(od, names[f])).reshape(-1)
    if f == "nacon":
      return int(a[0])
    return a.reshape(-1, shapes[f]) if f in shapes else a

  _check_contact(case, get)


def test_pair_margin_box_box_refused():
  import mujoco_warp_amd as mjw

  mjm = mjcf.load_model_from_string(KAT["refuse_margin_box_box"])
  with pytest.raises(NotImplementedError):
    mjw.put_model(mjm, device="cpu")


def test_pair_defaults_from_geoms():
  """Attributes a <pair> leaves unset come from its geoms (MuJoCo's compiler, mjCPair::Compile): margin /
  gap max, equal priority -> max condim and friction, solmix-weighted solref / solimp.  Parity unpinned:
  the rule is MuJoCo's compiler, which no reference test exercises."""
  mjm = mjcf.load_model_from_string("""
    <mujoco><worldbody>
      <body><freejoint/><geom name="a" size=".1" margin=".01" gap=".002" condim="4" friction="1 .02 .003"
         solmix="3" solref=".04 2" solimp=".8 .9 .01 .5 2"/></body>
      <body pos="0 0 .3"><freejoint/><geom name="b" size=".1" margin=".03" condim="1" friction=".5 .05 .001"
         solmix="1" solref=".02 1"/></body>
    </worldbody><contact><pair geom1="a" geom2="b"/></contact></mujoco>""")
  assert mjm.npair == 1 and mjm.pair_dim[0] == 4
  np.testing.assert_allclose(mjm.pair_margin, [0.03])
  np.testing.assert_allclose(mjm.pair_gap, [0.002])
  np.testing.assert_allclose(mjm.pair_friction[0], [1, 1, 0.05, 0.003, 0.003])
  np.testing.assert_allclose(mjm.pair_solref[0], [0.75 * 0.04 + 0.25 * 0.02, 0.75 * 2 + 0.25 * 1])
  np.testing.assert_allclose(mjm.pair_solimp[0], 0.75 * np.array([0.8, 0.9, 0.01, 0.5, 2]) + 0.25 * np.array([0.9, 0.95, 0.001, 0.5, 2]))
  np.testing.assert_allclose(mjm.pair_solreffriction[0], [0, 0])


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=IDS)
def test_hip_contact_pair_kat(case):
  import torch

  import mujoco_warp_amd as mjw

  mjm = mjcf.load_model_from_string(case["xml"])
  m = mjw.put_model(mjm, device="cuda")
  _check_pairid(case, mjm)
  np.testing.assert_array_equal(m.nxn_pairid.cpu().numpy(), nxn_geom_pairs(mjm, unfiltered=True)[1])
  d = mjw.make_data(mjm, nworld=1, nconmax=16, njmax=64, device="cuda", m=m)
  mjw.fwd_position(m, d)
  torch.cuda.synchronize()

  def get(f):
    if f == "nacon":
      return int(d.nacon[0])
    return getattr(d.contact, f).cpu().numpy()

  _check_contact(case, get)


_ROLLOUT = """
<mujoco>
  <option cone="{cone}"/>
  <worldbody>
    <geom name="floor" type="plane" size="2 2 .1" contype="0" conaffinity="0"/>
    <body pos="0 0 .1"><freejoint/><geom name="ball" size=".1" margin=".02" contype="0" conaffinity="0"/></body>
    <body pos=".25 0 .05"><freejoint/><geom name="ball2" type="capsule" size=".05 .1" euler="0 90 0"/></body>
    <geom name="ground2" type="plane" size="2 2 .1"/>
  </worldbody>
  <contact>
    <pair geom1="floor" geom2="ball" condim="6" friction=".8 .6 .01 .002 .001" solref=".03 1.2"
          solreffriction=".05 1" solimp=".85 .95 .002 .5 2" margin=".02" gap=".005"/>
  </contact>
</mujoco>"""


@pytest.mark.gpu
@pytest.mark.parametrize("cone", ["pyramidal", "elliptic"])
def test_hip_pair_rollout_matches_oracle(cone):
  """A sphere held by an explicit condim-6 pair (anisotropic friction, solreffriction, margin / gap) next to
  a capsule on an ordinary geom pair: 20 steps on the HIP path against the fp64 oracle.  The ball's own geom
  margin lets it pass the broadphase, which (as in the reference) tests geom margins, not the pair's."""
  import torch

  import mujoco_warp_amd as mjw
  from oracle import orc

  mjm = mjcf.load_model_from_string(_ROLLOUT.format(cone=cone))
  nworld, nstep = 4, 20
  rng = np.random.default_rng(3)
  qvel0 = rng.normal(scale=0.05, size=(nworld, mjm.nv))
  m = mjw.put_model(mjm, device="cuda")
  d = mjw.make_data(mjm, nworld=nworld, nconmax=32, njmax=64, device="cuda", m=m)
  d.qvel[:] = torch.as_tensor(qvel0, dtype=torch.float32, device="cuda")
  om = orc.OracleModel(mjm)
  od = orc.OracleData(om, nworld, 64, 32)
  od.qpos[:] = np.tile(mjm.qpos0, (nworld, 1))
  od.qvel[:] = qvel0
  for _ in range(nstep):
    mjw.step(m, d)
    od.step()
  torch.cuda.synchronize()
  assert int(d.nacon[0]) == int(np.sum(od.ncon)) == 3 * nworld  # the pair contact + 2 capsule contacts
  qpos, qvel = d.qpos.cpu().numpy(), d.qvel.cpu().numpy()
  # the ball on its explicit pair: tight
  np.testing.assert_allclose(qpos[:, :7], od.qpos[:, :7], atol=2e-5)
  assert np.linalg.norm(qvel[:, :6] - od.qvel[:, :6]) <= 1e-3 * max(1.0, np.linalg.norm(od.qvel[:, :6]))
  # the capsule's two frictional contacts are ill-conditioned: the fp32 oracle itself departs from the fp64
  # one by 1.5e-4 in x and 3e-4 in the quaternion over these 20 steps, so it gets that spread
  np.testing.assert_allclose(qpos[:, 7:], od.qpos[:, 7:], atol=1e-3)
