"""Diagnostic: sparse / flex pipeline (csrc/mjw_sparse.hip) vs the fp64 oracle on the cloth scene
(or aloha_cloth).

Prints the worst relative error per stage instead of asserting, so one GPU call shows every
mismatch.  Usage: python tools/cloth_diag.py [nworld] [nstep] [cloth|aloha]
"""

import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tests.cloth_common import cloth_model, cloth_states, dense_J, dense_qM, gpu_contacts, oracle_contacts  # noqa: E402
from tests.common import gpu_from_state, np_, oracle_from_state  # noqa: E402


def rel(a, b):
  a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
  if a.shape != b.shape:
    return f"shape {a.shape} vs {b.shape}"
  if a.size == 0:
    return "empty"
  err = np.abs(a - b)
  scale = np.maximum(np.abs(b), 1e-3 * max(1.0, np.abs(b).max()))
  i = np.unravel_index(np.argmax(err / scale), err.shape)
  return f"max|d| {err.max():.3e}  max rel {float((err / scale)[i]):.3e} at {i} (got {a[i]:.6g} want {b[i]:.6g})"


def main():
  import torch

  import mujoco_warp_amd as mjw

  nworld = int(sys.argv[1]) if len(sys.argv) > 1 else 2
  nstep = int(sys.argv[2]) if len(sys.argv) > 2 else 3
  which = sys.argv[3] if len(sys.argv) > 3 else "cloth"
  if which == "aloha":
    from tests.cloth_common import aloha_model, aloha_states

    mjm = aloha_model()
    qpos, qvel, ctrl = aloha_states(mjm, nworld, seed=0)
    njmax, nconmax = 16384, 4096
  else:
    mjm = cloth_model()
    qpos, qvel, ctrl = cloth_states(mjm, nworld, seed=0)
    njmax, nconmax = 3000, 200
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=njmax, nconmax=nconmax)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=njmax, nconmax=nconmax)
  t = time.time()
  mjw.fwd_position(m, d)
  torch.cuda.synchronize()
  print("gpu fwd_position", time.time() - t, flush=True)
  od.fwd_position()
  nv = mjm.nv
  for w in range(nworld):
    print(f"--- world {w}: ne {int(d.ne[w])}/{int(od.ne[w,0])} nf {int(d.nf[w])}/{int(od.nf[w,0])} nl {int(d.nl[w])}/{int(od.nl[w,0])} "
          f"nefc {int(d.nefc[w])}/{int(od.nefc[w,0])}", flush=True)
    for f in ("xpos", "xquat", "geom_xpos", "subtree_com", "cdof", "cinert", "crb", "flexvert_xpos", "flexedge_length", "flexedge_J"):
      print(f"  {f:16s}", rel(np_(getattr(d, f)[w]).ravel(), getattr(od, f)[w].ravel()))
    print("  qM              ", rel(dense_qM(mjm, np_(d.qM[w])), od.qM[w].reshape(nv, nv)))
    gc, oc = gpu_contacts(d, w), oracle_contacts(od, w)
    print(f"  ncon {len(gc)}/{len(oc)}")
    if len(gc) == len(oc) and len(gc):
      for k in ("dist", "pos", "frame"):
        print(f"  con_{k:12s}", rel(np.array([c[k] for c in gc]), np.array([c[k] for c in oc])))
    n = min(int(d.nefc[w]), int(od.nefc[w, 0]), njmax)
    if n:
      tg = d.efc.type[w, :n].cpu().numpy()
      to = od.efc_type[w, :n]
      print("  efc types equal", bool((tg == to).all()), "ids equal", bool((d.efc.id[w, :n].cpu().numpy() == od.efc_id[w, :n]).all()))
      print("  J               ", rel(dense_J(d, w, n, nv), od.efc_J[w].reshape(njmax, nv)[:n]))
      for f in ("pos", "D", "aref", "vel"):
        print(f"  efc_{f:12s}", rel(np_(getattr(d.efc, f)[w, :n]), getattr(od, "efc_" + f)[w, :n]))
  t = time.time()
  mjw.forward(m, d)
  torch.cuda.synchronize()
  print("gpu forward", time.time() - t, flush=True)
  od.forward()
  for f in ("qfrc_passive", "qfrc_bias", "qacc_smooth", "qacc", "qfrc_constraint"):
    print(f"  {f:16s}", rel(np_(getattr(d, f)), getattr(od, f)))
  print("  niter", d.solver_niter.cpu().numpy().ravel().tolist(), od.solver_niter.ravel().tolist())
  m2, d2 = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=njmax, nconmax=nconmax)
  om2, od2 = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=njmax, nconmax=nconmax)
  for s in range(nstep):
    mjw.step(m2, d2)
    od2.step()
    torch.cuda.synchronize()
    print(f"step {s}: qpos", rel(np_(d2.qpos), od2.qpos), " qvel", rel(np_(d2.qvel), od2.qvel), flush=True)
  # timing
  m3, d3 = gpu_from_state(mjm, np.repeat(qpos[:1], 256, 0), np.repeat(qvel[:1], 256, 0), np.repeat(ctrl[:1], 256, 0), njmax=njmax, nconmax=nconmax)
  print("ncollision", int(d.ncollision), "nacon", int(d.nacon))
  for _ in range(3):
    mjw.step(m3, d3)
  torch.cuda.synchronize()
  t = time.time()
  for _ in range(10):
    mjw.step(m3, d3)
  torch.cuda.synchronize()
  dt = (time.time() - t) / 10
  print(f"nworld 256: {dt*1e3:.2f} ms/step, {256/dt:.0f} env-steps/s; nan worlds {int(torch.isnan(d3.qpos).any(1).sum())}")


if __name__ == "__main__":
  main()
