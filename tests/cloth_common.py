"""Cloth-scene helpers for the sparse / flex parity tests (test infrastructure only).

The scene is the reference's `benchmarks/cloth/scene.xml` (a static-joint mannequin under a 30x30
dim-2 flexcomp towel), copied under models/cloth/.  States lower the towel onto the mannequin's head
and shoulders so that flex-geom contacts exist from the first step.
"""

from __future__ import annotations

import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLOTH = os.path.join(ROOT, "models", "cloth", "scene.xml")


def cloth_model():
  from mujoco_warp_amd import mjcf

  return mjcf.load_model(CLOTH)


ALOHA = os.path.join(ROOT, "models", "aloha_cloth", "scene.xml")


def aloha_model():
  from mujoco_warp_amd import mjcf

  return mjcf.load_model(ALOHA)


def aloha_states(mjm, nworld, seed=0, qnoise=0.05, vnoise=0.1):
  """Keyframe 0 (neutral pose, towel on the table) with seeded arm joint / velocity noise."""
  from mujoco_warp_amd import mjcf

  rng = np.random.default_rng(seed)
  d = mjcf.MjData(mjm)
  mjcf.reset_data_keyframe(mjm, d, 0)
  qpos = np.tile(d.qpos, (nworld, 1))
  na = 16  # the two arms' joints come first (the flexcomp's slide joints follow)
  qpos[:, :na] += rng.normal(0, qnoise, (nworld, na)) * (np.arange(na) % 8 < 6)
  qvel = np.zeros((nworld, mjm.nv))
  qvel[:, :na] = rng.normal(0, vnoise, (nworld, na))
  ctrl = np.tile(d.ctrl, (nworld, 1))
  return qpos, qvel, ctrl


def flex_vert_adr(mjm, kind="qpos"):
  """(nflexvert, 3) qpos (or dof) addresses of the slide joints that carry each flex vertex."""
  out = np.full((mjm.nflexvert, 3), -1, dtype=np.int64)
  src = mjm.jnt_qposadr if kind == "qpos" else mjm.jnt_dofadr
  for v in range(mjm.nflexvert):
    b = mjm.flex_vertbodyid[v]
    if mjm.body_jntnum[b] == 3:
      a = src[mjm.body_jntadr[b]]
      out[v] = [a, a + 1, a + 2]
  return out


def cloth_states(mjm, nworld, seed=0, dz=-0.43, vnoise=0.05):
  """Towel lowered by `dz` (onto the mannequin), small per-world vertex velocities (seeded)."""
  rng = np.random.default_rng(seed)
  qpos = np.tile(mjm.qpos0, (nworld, 1))
  adr = flex_vert_adr(mjm)
  adr = adr[adr[:, 0] >= 0]
  qpos[:, adr[:, 2]] += dz
  qpos[:, adr[:, :2]] += rng.normal(0, 0.002, (nworld, len(adr), 2))
  dadr = flex_vert_adr(mjm, "dof")
  dadr = dadr[dadr[:, 0] >= 0]
  qvel = np.zeros((nworld, mjm.nv))
  qvel[:, dadr.ravel()] = rng.normal(0, vnoise, (nworld, dadr.size))
  return qpos, qvel, np.zeros((nworld, mjm.nu))


def dense_qM(mjm, qm_sparse):
  """Sparse ancestor-row qM (M_rowadr / M_colind, diagonal last) -> dense symmetric (nv, nv)."""
  nv = mjm.nv
  M = np.zeros((nv, nv))
  for i in range(nv):
    a, n = mjm.M_rowadr[i], mjm.M_rownnz[i]
    for k in range(n):
      j = mjm.M_colind[a + k]
      M[i, j] = M[j, i] = qm_sparse[a + k]
  return M


def dense_J(d, w, n, nv):
  """First n sparse efc rows of world w (slot-major efc_J values / colind, rownnz) -> dense (n, nv)."""
  vals = d.efc.J[w, :, :n].detach().cpu().numpy().astype(np.float64)
  cols = d.efc.J_colind[w, :, :n].cpu().numpy()
  nnz = d.efc.J_rownnz[w, :n].cpu().numpy()
  J = np.zeros((n, nv))
  for r in range(n):
    for k in range(nnz[r]):
      J[r, cols[k, r]] += vals[k, r]
  return J


def _con_key(c):
  return (c["geom"][0], c["geom"][1], c["flex"][0], c["flex"][1], c["vert"][0], c["vert"][1], round(float(c["pos"][0]), 4), round(float(c["pos"][1]), 4))


def gpu_contacts(d, w):
  """Contacts of world w from the device pool, sorted by (geoms, flexes, verts, pos)."""
  start, cnt = (int(x) for x in d.ncon_world[w].cpu().numpy())
  out = []
  for s in range(start, start + cnt):
    out.append(dict(
      dist=float(d.contact.dist[s]), pos=d.contact.pos[s].cpu().numpy().astype(np.float64),
      frame=d.contact.frame[s].cpu().numpy().astype(np.float64).ravel(), geom=tuple(int(x) for x in d.contact.geom[s]),
      flex=tuple(int(x) for x in d.contact.flex[s]), vert=tuple(int(x) for x in d.contact.vert[s]), dim=int(d.contact.dim[s]), slot=s))
  return sorted(out, key=_con_key)


def oracle_contacts(od, w):
  n = min(int(od.ncon[w, 0]), od.nconmax)
  out = []
  for c in range(n):
    out.append(dict(
      dist=float(od.con_dist[w, c]), pos=od.con_pos[w, 3 * c : 3 * c + 3].copy(), frame=od.con_frame[w, 9 * c : 9 * c + 9].copy(),
      geom=tuple(int(x) for x in od.con_geom[w, 2 * c : 2 * c + 2]), flex=tuple(int(x) for x in od.con_flex[w, 2 * c : 2 * c + 2]),
      vert=tuple(int(x) for x in od.con_vert[w, 2 * c : 2 * c + 2]), dim=int(od.con_dim[w, c]), slot=c))
  return sorted(out, key=_con_key)
