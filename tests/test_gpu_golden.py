"""The HIP collision code against the reference's own collision known-answer tests (GPU).

Same cases as tests/test_golden.py (oracle), replayed on the device code the step runs: the
mjw_ccd.h GJK / EPA / box multi-contact (one wavefront per case over an LDS workspace) and the
mjw_flexcol.h triangle narrowphase, through the C ABI entry point mjw_kat (csrc/mjw_kat.hip).
Checks are the reference tests' own assertions (collision_gjk_test.py / collision_primitive_core_test.py).
"""

import numpy as np
import pytest
import torch

import golden_kat as gk

KAT = gk.load()
pytestmark = pytest.mark.gpu

CCD_IN, CCD_OUT, TRI_IN, TRI_OUT = 48, 8, 32, 16


def _kat(which, recs, aux, nout):
  from mujoco_warp_amd import _lib

  L = _lib.lib()
  dev = torch.device("cuda", 0)
  x = torch.as_tensor(np.ascontiguousarray(recs, np.float32).reshape(-1), device=dev)
  a = torch.as_tensor(np.ascontiguousarray(aux, np.float32).reshape(-1), device=dev)
  out = torch.zeros(len(recs) * nout, dtype=torch.float32, device=dev)
  stream = torch.cuda.current_stream(dev).cuda_stream
  _lib.check(L.mjw_kat(which, x.data_ptr(), a.data_ptr(), out.data_ptr(), len(recs), stream), "mjw_kat")
  torch.cuda.synchronize()
  return out.cpu().numpy().reshape(len(recs), nout)


def _ccd_record(a, vert_base):
  r = np.zeros(CCD_IN, np.float32)
  r[0:2] = a["types"]
  r[2:5], r[5:14], r[14:17] = a["pos"][0], a["mat"][0], a["size"][0]
  r[17:20], r[20:29], r[29:32] = a["pos"][1], a["mat"][1], a["size"][1]
  r[32], r[33], r[34], r[35] = a["margin"], a["tolerance"], a["iterations"], float(a["multiccd"])
  r[36], r[37], r[38], r[39] = a["vertadr"][0] + vert_base, a["vertnum"][0], a["vertadr"][1] + vert_base, a["vertnum"][1]
  return r


@pytest.fixture(scope="module")
def gjk_results():
  """All GJK cases in one launch (one wavefront each); mesh vertices of every scene concatenated."""
  cases = [c for c in KAT["gjk"] if c["name"] not in gk.UNSUPPORTED and c["name"] not in gk.DEVICE_PIPELINE_ONLY]
  recs, verts, base = [], [], 0
  for c in cases:
    a = gk.gjk_inputs(c)
    recs.append(_ccd_record(a, base))
    verts.append(a["mesh_vert"])
    base += len(a["mesh_vert"])
  max_it = max(int(r[34]) for r in recs)
  aux = np.concatenate([[max_it], np.concatenate(verts).reshape(-1)])
  out = _kat(0, np.stack(recs), aux, CCD_OUT)
  return {c["name"]: out[i] for i, c in enumerate(cases)}


@pytest.mark.parametrize("case", KAT["gjk"], ids=[c["name"] for c in KAT["gjk"]])
def test_hip_gjk_kat(case, gjk_results):
  if case["name"] in gk.UNSUPPORTED:
    pytest.skip(gk.UNSUPPORTED[case["name"]])
  if case["name"] in gk.DEVICE_PIPELINE_ONLY:
    pytest.skip(gk.DEVICE_PIPELINE_ONLY[case["name"]])
  o = gjk_results[case["name"]]
  assert o[0] >= 0
  gk.check(case, dict(ncon=int(o[0]), dist=float(o[1]), x1=o[2:5].astype(np.float64), x2=o[5:8].astype(np.float64)))


@pytest.fixture(scope="module")
def tri_results():
  recs = []
  for c in KAT["triangle"]:
    gt, gp, gr, gs, t, tr = gk.triangle_inputs(c)
    r = np.zeros(TRI_IN, np.float32)
    r[0], r[1:4], r[4:13], r[13:16], r[16:25], r[25] = gt, gp, gr, gs, np.asarray(t).reshape(9), tr
    recs.append(r)
  out = _kat(1, np.stack(recs), np.zeros(1), TRI_OUT)
  return {c["name"]: out[i] for i, c in enumerate(KAT["triangle"])}


@pytest.mark.parametrize("case", KAT["triangle"], ids=[c["name"] for c in KAT["triangle"]])
def test_hip_triangle_kat(case, tri_results):
  o = tri_results[case["name"]]
  c2 = o[1:15].reshape(2, 7).astype(np.float64)
  if case["kind"] == "sphere":
    res = dict(dist=c2[0, 0], pos=c2[0, 1:4], normal=c2[0, 4:7])
  else:
    res = dict(dist=c2[:, 0], pos=c2[:, 1:4], normal=c2[:, 4:7])
  gk.check(case, res)


def test_hip_matches_fp32_oracle_kat(gjk_results):
  """Beyond the reference's assertions: the device result equals the fp32 oracle's to fp32 round-off
  (dist within 1e-6 absolute or 1e-4 relative, same contact count) on every extracted GJK case."""
  from oracle import orc

  for c in KAT["gjk"]:
    if c["name"] in gk.UNSUPPORTED or c["name"] in gk.DEVICE_PIPELINE_ONLY:
      continue
    a = gk.gjk_inputs(c)
    n, d, _, _ = orc.kat_ccd(a["types"], a["pos"], a["mat"], a["size"], a["margin"], a["tolerance"], a["iterations"], a["multiccd"],
                             a["mesh_vert"], a["vertadr"], a["vertnum"], real_bits=32)
    o = gjk_results[c["name"]]
    assert int(o[0]) == n, c["name"]
    assert abs(o[1] - d) <= max(1e-6, 1e-4 * abs(d)), (c["name"], o[1], d)


@pytest.mark.parametrize("case", KAT["broadphase"], ids=[f"{c['source']}-f{c['filter']}-k{c['keys']}" for c in KAT["broadphase"]])
def test_hip_broadphase_kat(case):
  """NXN broadphase pair counts of broadphase_test.py on the forward kernel (d.ncollision after
  fwd_position): plane / sphere / AABB / OBB filter combinations, margins, filterparent, contype."""
  import mujoco_warp_amd as mjw

  mjm, qpos = gk.broadphase_model(case)
  m = mjw.put_model(mjm, device="cuda")
  m.opt.broadphase_filter = int(case["filter"])
  d = mjw.make_data(mjm, nworld=len(qpos), nconmax=16, njmax=64, device="cuda", m=m)
  d.qpos[:] = torch.as_tensor(qpos, dtype=torch.float32, device="cuda")
  mjw.fwd_position(m, d)
  torch.cuda.synchronize()
  assert int(d.ncollision[0]) == case["ncollision"], case["source"]
