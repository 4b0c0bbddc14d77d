"""Inputs and checks of the reference's collision known-answer tests (tests/golden/collision_kat.json).

`gjk_inputs(case)` compiles the case's MJCF literal with this build's compiler and returns the two geoms
exactly as the reference's `_geom_dist` helper hands them to `ccd()` (collision_gjk_test.py:34-265):
type, world pose (the literal pos/mat when the test gives one, else the compiled worldbody geom frame),
size, mesh vertices, margin, opt.ccd_tolerance and opt.ccd_iterations.  `check(case, results)` applies
the test's own assertions with unittest's semantics (assertAlmostEqual: round(a - b, places) == 0).
"""

from __future__ import annotations

import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
KAT = os.path.join(HERE, "golden", "collision_kat.json")

# every case runs (mesh multi-contact: the compiler's mesh polygon data, mjcf._mesh_polygons); the device
# KAT kernel replays the primitive / box cases, and tests/test_multiccd.py runs the mesh case through the
# device pipeline
UNSUPPORTED = {}
# cases the device KAT kernel (csrc/mjw_kat.hip, no model: no mesh polygon data) leaves to the pipeline test
DEVICE_PIPELINE_ONLY = {"test_mesh_mesh_ccd": "mesh multi-contact: run through the device pipeline (tests/test_multiccd.py)"}

# cases whose expected value is the reference's own fp32 (Warp `float`) result rather than MuJoCo C's
# fp64 one: the fp64 oracle lands elsewhere and is not held to them (fp32 oracle and HIP are).
#   test_box_box_max  : fp64 depth -0.0363624014, the fp32 value -0.03636224 differs in the 7th place
#   test_box_box_max2 : "GJK converges very slowly" -- in fp32 GJK stops 1.39e-6 outside the tolerance
#                       (separated); in fp64 it converges and EPA finds a 4.9e-5 penetration
FP32_ONLY = {"test_box_box_max", "test_box_box_max2"}


def load():
  with open(KAT) as f:
    return json.load(f)


def gjk_inputs(case):
  import mujoco_warp_amd as mjw
  from mujoco_warp_amd.mjcf import quat_to_mat

  mjm = mjw.load_model_from_string(case["xml"])
  if case["overrides"]:
    mjw.override_model(mjm, case["overrides"])
  gids = (case["gid1"], case["gid2"])
  types = np.array([mjm.geom_type[g] for g in gids], np.int32)
  pos = np.zeros((2, 3))
  mat = np.zeros((2, 9))
  for k, g in enumerate(gids):
    assert mjm.geom_bodyid[g] == 0, "KAT scenes place their geoms in the worldbody"
    pos[k] = case.get(f"pos{k + 1}", mjm.geom_pos[g])
    mat[k] = case.get(f"mat{k + 1}", np.asarray(quat_to_mat(mjm.geom_quat[g])).reshape(9))
  size = np.array([mjm.geom_size[g] for g in gids], np.float64)
  vertadr = np.zeros(2, np.int32)
  vertnum = np.zeros(2, np.int32)
  for k, g in enumerate(gids):
    if types[k] == 7:  # mesh
      mid = mjm.geom_dataid[g]
      vertadr[k], vertnum[k] = mjm.mesh_vertadr[mid], mjm.mesh_vertnum[mid]
  mesh_vert = np.asarray(mjm.mesh_vert, np.float64).reshape(-1, 3) if mjm.nmesh else np.zeros((1, 3))
  meshid = np.array([mjm.geom_dataid[g] if types[k] == 7 else -1 for k, g in enumerate(gids)], np.int32)
  return dict(types=types, pos=pos, mat=mat, size=size, mesh_vert=mesh_vert, vertadr=vertadr, vertnum=vertnum,
              margin=case["margin"], tolerance=float(mjm.opt.ccd_tolerance), iterations=int(mjm.opt.ccd_iterations),
              multiccd=case["multiccd"], mjm=mjm, meshid=meshid)


def triangle_inputs(case):
  """(geom type, pos, rot, size, triangle[3, 3], tri_radius) of a collision_primitive_core_test case;
  capsule / cylinder axes go in column 2 of the rotation (the narrowphase reads the geom z-axis)."""
  kind = case["kind"]
  t = np.asarray(case["t"], np.float64)
  gp = np.asarray(case["center"], np.float64)
  if kind == "sphere":
    return 2, gp, np.eye(3).reshape(9), np.array([case["radius"], 0, 0]), t, case["tri_radius"]
  if kind == "box":
    return 6, gp, np.asarray(case["rot"], np.float64), np.asarray(case["size"], np.float64), t, case["tri_radius"]
  ax = np.asarray(case["axis"], np.float64)
  rot = np.zeros((3, 3))
  rot[:, 2] = ax
  gt = 3 if kind == "capsule" else 5
  return gt, gp, rot.reshape(9), np.array([case["radius"], case["half"], 0]), t, case["tri_radius"]


def _value(res, q, idx):
  v = res[q]
  if idx is not None:
    v = np.asarray(v)[idx]
  return v


def check(case, res):
  """Apply the reference test's assertions to `res` (dict of dist / ncon / x1 / x2 / normal / pos)."""
  if "x1" in res and "x2" in res:
    diff = np.asarray(res["x1"], np.float64) - np.asarray(res["x2"], np.float64)
    n = np.linalg.norm(diff)
    res = dict(res, normal=diff / n if n > 0 else diff)
  for c in case["checks"]:
    got = _value(res, c["quantity"], c["index"])
    want = c["value"]
    where = f"{case['name']} ({case['source']}, check at line {c['line']}): {c['quantity']}"
    if c["op"] == "eq":
      assert got == want, f"{where} = {got!r}, reference asserts == {want!r}"
    elif c["op"] == "almost":
      assert round(abs(float(got) - float(want)), c["places"]) == 0, f"{where} = {float(got)!r}, reference {want!r} to {c['places']} places"
    elif c["op"] == "lt":
      assert float(np.max(got)) < want, f"{where} = {got!r}, reference asserts < {want!r}"
    elif c["op"] == "gt":
      assert float(np.min(got)) > want, f"{where} = {got!r}, reference asserts > {want!r}"
    elif c["op"] == "allclose":
      np.testing.assert_allclose(got, want, atol=c["atol"], err_msg=where)
    else:
      raise AssertionError(f"unknown check {c}")


def broadphase_model(case):
  """Compiled scene of a broadphase_test.py case with its filter / disableflags / contype edits, and the
  per-world qpos of its keyframe(s)."""
  import mujoco_warp_amd as mjw

  mjm = mjw.load_model_from_string(case["xml"])
  mjm.opt.broadphase_filter = int(case["filter"])
  mjm.opt.disableflags = int(mjm.opt.disableflags) | int(case["disableflags"])
  if "geom_contype_first3" in case:
    mjm.geom_contype[:3] = case["geom_contype_first3"]
  qpos = np.stack([np.asarray(mjm.key_qpos[k], np.float64) for k in case["keys"]])
  return mjm, qpos
