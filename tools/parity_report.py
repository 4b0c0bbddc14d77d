"""Per-field error report of the HIP path against the fp64 oracle (GPU box; prints JSON).

For each Data field after each stage: `norm` = max|got - want| / scale with scale = max|want| over
the world (normwise relative error), and `elem` = the smallest elementwise rtol that passes with an
absolute floor of 1e-6 * scale (SURVEY.md 8(c) P0 rung).  Used to set the strict parity tests'
tolerances from measured data (tests/test_gpu_parity_strict.py).
usage: python tools/parity_report.py [out.json]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tests.common import gpu_from_state, humanoid_model, np_, oracle_from_state, random_states  # noqa: E402


def err(got, want):
  got = np.asarray(got, np.float64).reshape(got.shape[0], -1)
  want = np.asarray(want, np.float64).reshape(want.shape[0], -1)
  scale = np.abs(want).max(axis=1, keepdims=True) + 1e-30
  e = np.abs(got - want)
  norm = float((e / scale).max())
  elem = float((np.maximum(e - 1e-6 * scale, 0) / np.maximum(np.abs(want), 1e-30)).max())
  return dict(norm=norm, elem=elem)


def main():
  import torch

  import mujoco_warp_amd as mjw

  out = {}
  mjm = humanoid_model("CG")
  nv = mjm.nv
  qpos, qvel, ctrl = random_states(mjm, 32, seed=11)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl)
  stages = [("fwd_position", ("xpos", "xquat", "xmat", "xipos", "ximat", "xanchor", "xaxis", "geom_xpos", "geom_xmat", "subtree_com",
                              "cinert", "cdof", "crb", "cam_xpos", "cam_xmat", "light_xpos", "light_xdir", "actuator_length")),
            ("fwd_velocity", ("actuator_velocity", "cvel", "cdof_dot", "qfrc_spring", "qfrc_damper", "qfrc_passive", "qfrc_bias")),
            ("fwd_actuation", ("actuator_force", "qfrc_actuator")),
            ("fwd_acceleration", ("qfrc_smooth", "qacc_smooth"))]
  for st, fields in stages:
    getattr(mjw, st)(m, d)
    getattr(od, st)()
    torch.cuda.synchronize()
    for f in fields:
      out[f] = err(np_(getattr(d, f)).reshape(d.nworld, -1), getattr(od, f))
  # constraint rows (deterministic order, identical counts) and contact distances (sorted per world)
  nw = d.nworld
  rows = {f: [] for f in ("J", "D", "aref", "pos", "vel", "margin")}
  cd = []
  nacon = int(d.nacon[0])
  gw = np_(d.contact.worldid[:nacon]).astype(int)
  for w in range(nw):
    n = min(int(d.nefc[w]), d.njmax)
    assert n == int(od.nefc[w, 0])
    rows["J"].append((np_(d.efc.J[w, :n, :nv]).ravel(), od.efc_J[w].reshape(od.njmax, nv)[:n].ravel()))
    for f in ("D", "aref", "pos", "vel", "margin"):
      rows[f].append((np_(getattr(d.efc, f)[w, :n]), getattr(od, "efc_" + f)[w, :n]))
    sel = np.nonzero(gw == w)[0]
    cd.append((np.sort(np_(d.contact.dist[:nacon])[sel]), np.sort(od.con_dist[w, : int(od.ncon[w, 0])])))
  for f, pairs in rows.items():
    e = [err(g[None], o[None]) for g, o in pairs if len(o)]
    out["efc_" + f] = dict(norm=max(x["norm"] for x in e), elem=max(x["elem"] for x in e))
  e = [err(g[None], o[None]) for g, o in cd if len(o)]
  out["contact_dist"] = dict(norm=max(x["norm"] for x in e), elem=max(x["elem"] for x in e))
  out["qM"] = err(np_(d.qM)[:, :nv, :nv].reshape(d.nworld, -1), od.qM)
  out["qLD"] = err(np_(d.qLD).reshape(d.nworld, -1), od.qLD)
  # backward error of qacc_smooth: |M64 qacc32 - f64| / |f64|
  M = od.qM.reshape(-1, nv, nv)
  r = np.einsum("wij,wj->wi", M, np_(d.qacc_smooth)) - od.qfrc_smooth
  out["qacc_smooth_backward"] = float((np.abs(r).max(axis=1) / np.abs(od.qfrc_smooth).max(axis=1)).max())
  # one contact-free step from key no_efc with random velocities / controls
  k = mjm.key_names.index("no_efc")
  qpos, qvel, ctrl = random_states(mjm, 16, seed=12, key=k, qpos_noise=0.02, qvel_noise=0.2)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl)
  mjw.step(m, d)
  od.step()
  torch.cuda.synchronize()
  out["no_efc_nefc"] = int(np_(d.nefc).max())
  for f in ("qpos", "qvel", "qacc"):
    out["no_efc_step_" + f] = err(np_(getattr(d, f)), getattr(od, f))
  js = json.dumps(out, indent=1)
  print(js)
  if len(sys.argv) > 1:
    with open(sys.argv[1], "w") as fh:
      fh.write(js)


if __name__ == "__main__":
  main()
