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

  Follows mj_setState's layout.  Two quirks of the reference kernel are not reproduced: it advances
  the read address by neq - 1 after EQ_ACTIVE (support.py:801, `adr += j`) and swaps the x / y
  components of MOCAP_POS (support.py:806-808); here every element is read at its mj_stateSize
  offset, so get_state / set_state round-trip exactly."""
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
  """6D force:torque of contacts (support.py:241-351), pyramidal decoding, optional world frame."""
  if m.opt.cone != ConeType.PYRAMIDAL:
    raise NotImplementedError("elliptic cones are not supported by this build")
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


def mul_m(m: Model, d: Data, res: torch.Tensor, vec: torch.Tensor, skip: Optional[torch.Tensor] = None, M: Optional[torch.Tensor] = None):
  """res = qM @ vec per world (support.py:132-171, dense qM)."""
  if M is None:
    M = d.qM
  nv = m.nv
  out = torch.bmm(M[:, :nv, :nv], vec.unsqueeze(-1)).squeeze(-1)
  if skip is None:
    res[:] = out
  else:
    keep = ~skip.to(torch.bool)
    res[keep] = out[keep]
