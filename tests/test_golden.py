"""The oracle against the reference's own collision known-answer tests (CPU).

Vectors: tests/golden/collision_kat.json, extracted as data from collision_gjk_test.py and
collision_primitive_core_test.py by tests/golden/make_golden_collision.py.  The same cases run on the
HIP path in tests/test_gpu_golden.py.
"""

import pytest

import golden_kat as gk
from oracle import orc

KAT = gk.load()


@pytest.mark.parametrize("real_bits", [64, 32])
@pytest.mark.parametrize("case", KAT["gjk"], ids=[c["name"] for c in KAT["gjk"]])
def test_oracle_gjk_kat(case, real_bits):
  if case["name"] in gk.UNSUPPORTED:
    pytest.skip(gk.UNSUPPORTED[case["name"]])
  if real_bits == 64 and case["name"] in gk.FP32_ONLY:
    pytest.skip("expected value is the reference's fp32 result (golden_kat.FP32_ONLY)")
  a = gk.gjk_inputs(case)
  ncon, dist, x1, x2 = orc.kat_ccd(a["types"], a["pos"], a["mat"], a["size"], a["margin"], a["tolerance"], a["iterations"],
                                   a["multiccd"], a["mesh_vert"], a["vertadr"], a["vertnum"], real_bits=real_bits, mjm=a["mjm"],
                                   meshid=a["meshid"])
  assert ncon >= 0
  gk.check(case, dict(dist=dist, ncon=ncon, x1=x1, x2=x2))


@pytest.mark.parametrize("real_bits", [64, 32])
@pytest.mark.parametrize("case", KAT["triangle"], ids=[c["name"] for c in KAT["triangle"]])
def test_oracle_triangle_kat(case, real_bits):
  gt, gp, gr, gs, t, tr = gk.triangle_inputs(case)
  n, out = orc.kat_geom_triangle(gt, gp, gr, gs, t, tr, real_bits=real_bits)
  assert n >= 0
  if case["kind"] == "sphere":
    res = dict(dist=out[0, 0], pos=out[0, 1:4], normal=out[0, 4:7])
  else:
    res = dict(dist=out[:, 0], pos=out[:, 1:4], normal=out[:, 4:7])
  gk.check(case, res)


def test_kat_inventory():
  """Every GJK test of the reference file is extracted except the parameterized support-function one."""
  assert len(KAT["gjk"]) >= 19 and KAT["gjk_not_extracted"] == ["test_hfield_support"]
  assert len(KAT["triangle"]) == 16


def test_oracle_fp64_reproduces_mujoco_c():
  """The reference records MuJoCo C's fp64 answer next to one fp32 expectation
  (collision_gjk_test.py test_box_box_horizon: "dist = -0.00011579410621457821 - MJC 64 bit precision");
  the fp64 oracle reproduces it to 1e-15."""
  done = 0
  for case in KAT["gjk"]:
    for c in case["checks"]:
      if "mjc64" not in c:
        continue
      a = gk.gjk_inputs(case)
      _, dist, _, _ = orc.kat_ccd(a["types"], a["pos"], a["mat"], a["size"], a["margin"], a["tolerance"], a["iterations"],
                                  a["multiccd"], a["mesh_vert"], a["vertadr"], a["vertnum"], real_bits=64)
      assert abs(dist - c["mjc64"]) < 1e-15, (case["name"], dist, c["mjc64"])
      done += 1
  assert done >= 1


@pytest.mark.parametrize("case", KAT["broadphase"], ids=[f"{c['source']}-f{c['filter']}-k{c['keys']}" for c in KAT["broadphase"]])
def test_oracle_broadphase_kat(case):
  """NXN broadphase pair counts of broadphase_test.py (filters, margins, filterparent, contype)."""
  import numpy as np

  mjm, qpos = gk.broadphase_model(case)
  om = orc.OracleModel(mjm)
  od = orc.OracleData(om, len(qpos), 64, 64)
  od.qpos[:] = qpos
  od.fwd_position()
  assert int(np.sum(od.ncollision)) == case["ncollision"], case["source"]
