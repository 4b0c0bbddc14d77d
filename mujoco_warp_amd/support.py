"""Support functions of the reference API on the device tensors (mirror mujoco_warp/_src/support.py).

State packing (`get_state` / `set_state`, support.py:572-830), contact forces (`contact_force`,
support.py:241-351) and `mul_m` (support.py:132-171).  These are gathers / scatters / small
reductions over Data fields that already live in HBM; they run as torch ops on the same device and
stream as the HIP kernels (no host round trip, no CPU fallback).
"""

from __future__ import annotations

from typing import Optional

import torch

from .types import ConeType, Data, Model, State

# State element order and sizes (types.py:598-638, support.py:615-700)
_ELEMENTS = (
  (State.TIME, "time", lambda m: 1),
  (State.QPOS, "qpos", lambda m: m.nq),
  (State.QVEL, "qvel", lambda m: m.nv),
  (State.ACT, "act", lambda m: m.na),
  (State.WARMSTART, "qacc_warmstart", lambda m: m.nv),
  (State.CTRL, "ctrl", lambda m: m.nu),
  (State.QFRC_APPLIED, "qfrc_applied", lambda m: m.nv),
  (State.XFRC_APPLIED, "xfrc_applied", lambda m: 6 * m.nbody),
  (State.EQ_ACTIVE, "eq_active", lambda m: m.neq),
  (State.MOCAP_POS, "mocap_pos", lambda m: 3 * m.nmocap),
  (State.MOCAP_QUAT, "mocap_quat", lambda m: 4 * m.nmocap),
)


def state_size(m: Model, sig: int) -> int:
  """mj_stateSize: number of floats in the state selected by `sig`."""
  if sig >= (1 << State.NSTATE):
    raise ValueError(f"invalid state signature {sig} >= 2^mjNSTATE")
  return sum(n(m) for bit, _, n in _ELEMENTS if sig & bit)


def get_state(m: Model, d: Data, state: torch.Tensor, sig: int, active: Optional[torch.Tensor] = None):
  """Copy the state components selected by `sig` from `d` into `state` (nworld, size) (support.py:572-708)."""
  if sig >= (1 << State.NSTATE):
    raise ValueError(f"invalid state signature {sig} >= 2^mjNSTATE")
  parts = []
  for bit, name, n in _ELEMENTS:
    if sig & bit:
      t = getattr(d, name).reshape(d.nworld, -1).to(state.dtype)
      parts.append(t[:, : n(m)])
  if not parts:
    return
  packed = torch.cat(parts, dim=1)
  if active is None:
    state[:, : packed.shape[1]] = packed
  else:
    sel = active.to(torch.bool)
    state[sel, : packed.shape[1]] = packed[sel]


def set_state(m: Model, d: Data, state: torch.Tensor, sig: int, active: Optional[torch.Tensor] = None):
  """Copy the state components selected by `sig` from `state` into `d` (support.py:711-830).

  Follows mj_setState's layout, which is what the reference's own test asserts (support_test.py:144-180:
  set_state of mj_getState's vector reproduces every MjData field, eq_active and mocap_pos included).
  Two quirks of the reference kernel that this test does not reach (its model has no mocap bodies) are
  therefore not reproduced: it advances the read address by neq - 1 after EQ_ACTIVE (support.py:801,
  `adr += j`), which shifts the mocap elements that follow, and swaps the x / y components of
  MOCAP_POS (support.py:806-808).  Here every element is read at its mj_stateSize offset, so
  get_state / set_state round-trip exactly."""
  if sig >= (1 << State.NSTATE):
    raise ValueError(f"invalid state signature {sig} >= 2^mjNSTATE")
  sel = None if active is None else active.to(torch.bool)
  adr = 0
  for bit, name, n in _ELEMENTS:
    if not sig & bit:
      continue
    k = n(m)
    dst = getattr(d, name)
    src = state[:, adr : adr + k].reshape((d.nworld,) + tuple(dst.shape[1:])).to(dst.dtype)
    if bit == State.EQ_ACTIVE:
      src = (src != 0).to(dst.dtype)
    if sel is None:
      dst[:] = src
    else:
      dst[sel] = src[sel]
    adr += k


def contact_force(m: Model, d: Data, contact_ids: torch.Tensor, to_world_frame: bool, force: torch.Tensor):
  """6D force:torque of contacts (support.py:241-351): pyramidal decoding, or the elliptic rows directly
  (support.py:296-299); optional world frame."""
  ids = contact_ids.to(torch.long)
  nacon = int(d.nacon[0])
  valid = (ids >= 0) & (ids < min(nacon, d.naconmax))
  ids_c = ids.clamp(0, max(d.naconmax - 1, 0))
  dim = d.contact.dim[ids_c]
  adr = d.contact.efc_address[ids_c, 0].to(torch.long)
  wid = d.contact.worldid[ids_c].to(torch.long)
  mu = d.contact.friction[ids_c]
  efc = d.efc.force
  out = torch.zeros((ids.shape[0], 6), dtype=efc.dtype, device=efc.device)
  ok = valid & (adr >= 0)

  def f_at(a):
    inb = ok & (a < d.njmax)
    return torch.where(inb, efc[wid, a.clamp(0, d.njmax - 1)], torch.zeros_like(out[:, 0]))

  if m.opt.cone != ConeType.PYRAMIDAL:
    for i in range(int(m.nmaxcondim)):
      a = d.contact.efc_address[ids_c, i].to(torch.long) if i < d.contact.efc_address.shape[1] else adr
      use = ok & (i < dim) & (a >= 0)
      out[:, i] = torch.where(use, f_at(a.clamp(min=0)), out[:, i])
    out[~ok] = 0
    if to_world_frame:
      frame = d.contact.frame[ids_c]
      out = torch.cat([torch.einsum("ni,nij->nj", out[:, :3], frame), torch.einsum("ni,nij->nj", out[:, 3:], frame)], dim=1)
    force[:] = out
    return
  out[:, 0] = torch.where(dim == 1, f_at(adr), out[:, 0])
  for i in range(int(m.nmaxcondim) - 1 if m.nmaxcondim > 1 else 0):
    use = ok & (dim > 1) & (i < dim - 1)
    d1, d2 = f_at(adr + 2 * i), f_at(adr + 2 * i + 1)
    out[:, 0] = torch.where(use, out[:, 0] + d1 + d2, out[:, 0])
    out[:, i + 1] = torch.where(use, (d1 - d2) * mu[:, i], out[:, i + 1])
  out[~ok] = 0
  if to_world_frame:
    frame = d.contact.frame[ids_c]
    out = torch.cat([torch.einsum("ni,nij->nj", out[:, :3], frame), torch.einsum("ni,nij->nj", out[:, 3:], frame)], dim=1)
  force[:] = out


def _mulm_index(m: Model):
  """Gather lists of the symmetric product with the sparse ancestor-row qM (support.py:67-101's
  qM_mulm_rowadr / _col / _madr, padded to the longest row): for dof i, the entries of row i (its
  ancestors and the diagonal) and the entries M[k, i] of every descendant k.  Padding points at a zero
  column appended to vec.  Built once per Model on the host, kept on the device."""
  idx = getattr(m, "_mulm_idx", None)
  if idx is not None:
    return idx
  nv = int(m.nv)
  rowadr = m.M_rowadr.reshape(-1).cpu().tolist()
  rownnz = m.M_rownnz.reshape(-1).cpu().tolist()
  colind = m.M_colind.reshape(-1).cpu().tolist()
  ent = [[] for _ in range(nv)]
  for i in range(nv):
    for k in range(rownnz[i]):
      a = rowadr[i] + k
      j = colind[a]
      ent[i].append((j, a))
      if j != i:
        ent[j].append((i, a))
  K = max(1, max(len(e) for e in ent))
  nM = int(m.nM)
  col = torch.full((nv, K), nv, dtype=torch.long)
  madr = torch.full((nv, K), nM, dtype=torch.long)
  for i, e in enumerate(ent):
    for k, (j, a) in enumerate(sorted(e)):
      col[i, k], madr[i, k] = j, a
  dev = m.M_rowadr.device
  idx = (col.to(dev), madr.to(dev))
  m._mulm_idx = idx
  return idx


def mul_m(m: Model, d: Data, res: torch.Tensor, vec: torch.Tensor, skip: Optional[torch.Tensor] = None, M: Optional[torch.Tensor] = None):
  """res = qM @ vec per world (support.py:132-171): dense qM (nworld, nv_pad, nv_pad) as a batched
  matvec; sparse qM (nworld, nM) in the ancestor-row layout as a gather over each dof's row and column
  entries (mul_m_sparse, support.py:67-101), summed in a fixed order."""
  if M is None:
    M = d.qM
  nv = m.nv
  if m.is_sparse:
    col, madr = _mulm_index(m)
    nw = M.shape[0]
    Mz = torch.cat([M.reshape(nw, -1), M.new_zeros((nw, 1))], dim=1)
    vz = torch.cat([vec.reshape(nw, -1)[:, :nv], vec.new_zeros((nw, 1))], dim=1)
    out = (Mz[:, madr] * vz[:, col]).sum(dim=2)
  else:
    out = torch.bmm(M[:, :nv, :nv], vec.unsqueeze(-1)).squeeze(-1)
  if skip is None:
    res[:] = out
  else:
    keep = ~skip.to(torch.bool)
    res[keep] = out[keep]


def efc_J_csr(m: Model, d: Data, njmax_nnz: Optional[int] = None):
  """The sparse constraint Jacobian in the reference's CSR layout (io.py:940-943: `efc.J_rownnz`,
  `efc.J_rowadr` (nworld, njmax), `efc.J_colind` / `efc.J` (nworld, 1, njmax_nnz)), converted from this
  build's slot-major ELL rows (slot k of row r at `efc_J[w, k, r]`).  Rows are packed in
  row order; columns ascend within a row.  Rows past nefc have rownnz 0.  Returns
  (J_rownnz, J_rowadr, J_colind, J); a device-side conversion (torch ops), no host round trip."""
  if not m.is_sparse:
    raise ValueError("efc_J_csr: dense models keep efc.J as (nworld, njmax_pad, nv_pad), as the reference does")
  nw, njmax = d.nworld, d.njmax
  dev = d.efc.J.device
  nnz = (njmax_nnz or getattr(d, "njmax_nnz", None) or njmax * int(m.nv))
  nrow = torch.minimum(d.nefc.reshape(nw), torch.tensor(njmax, device=dev)).to(torch.long)
  rows = torch.arange(njmax, device=dev)
  rownnz = torch.where(rows[None, :] < nrow[:, None], d.efc.J_rownnz.reshape(nw, -1)[:, :njmax].to(torch.long), torch.zeros((), dtype=torch.long, device=dev))
  rowadr = torch.cumsum(rownnz, dim=1) - rownnz
  if int((rowadr[:, -1] + rownnz[:, -1]).max()) > nnz:
    raise ValueError(f"efc_J_csr: more than njmax_nnz = {nnz} non-zeros")
  njrow = d.efc.J.shape[1]
  vals = d.efc.J.reshape(nw, njrow, -1)[:, :, :njmax].transpose(1, 2)  # (nw, njmax, njrow)
  cols = d.efc.J_colind.reshape(nw, njrow, -1)[:, :, :njmax].transpose(1, 2).to(torch.long)
  slot = torch.arange(njrow, device=dev)
  valid = slot[None, None, :] < rownnz[:, :, None]
  big = int(m.nv) + 1
  key = torch.where(valid, cols, torch.full_like(cols, big))
  key, order = torch.sort(key, dim=2, stable=True)
  vals = torch.gather(vals, 2, order)
  pos = rowadr[:, :, None] + slot[None, None, :]
  wid = torch.arange(nw, device=dev)[:, None, None].expand_as(pos)
  J = torch.zeros((nw, 1, nnz), dtype=vals.dtype, device=dev)
  colind = torch.zeros((nw, 1, nnz), dtype=torch.int32, device=dev)
  J[wid[valid], 0, pos[valid]] = vals[valid]
  colind[wid[valid], 0, pos[valid]] = key[valid].to(torch.int32)
  return rownnz.to(torch.int32), rowadr.to(torch.int32), colind, J
