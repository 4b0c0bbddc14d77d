"""The reference's finer-grained stage and support functions, on this build's fused launches.

`mujoco_warp` exposes every pipeline stage as its own function (mujoco_warp/__init__.py:26-112:
`kinematics`, `com_pos`, `crb`, `collision`, `make_constraint`, `rne`, ...).  Here a stage group runs as
one HIP launch, so each of these functions runs the launch that contains it:

* position stage (`mjw_fwd_position`): kinematics, com_pos, camlight, flex, tendon, crb, collision,
  make_constraint, transmission -- each computes its reference outputs from `qpos` / `mocap_*` (and the
  stage's other outputs along with them; an input the reference would read from an earlier stage's output,
  e.g. a hand-edited `d.xipos` before `com_pos`, is recomputed from `qpos`, not taken from `d`);
* velocity stage (`mjw_fwd_velocity`): com_vel, passive, rne (flg_acc = False);
* `factor_m`: the acceleration stage launch, whose dense kernel factors qM into qLD
  (it also refreshes qfrc_smooth / qacc_smooth from the current force inputs);
* `rne_postconstraint`: the sensor kernel's acceleration stage (cacc, cfrc_int, cfrc_ext).

The support functions that take caller arrays -- `jac`, `xfrc_accumulate`, `solve_m`, `subtree_vel`,
`energy_pos`, `energy_vel` -- are torch ops on the Data tensors in HBM, on the device and stream of the
HIP launches (restatements of support.py / smooth.py / sensor.py, cited per function).  None of them is on
the `step` path.
"""

from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from .forward import _call, _sensor, fwd_position, fwd_velocity
from .types import Data, DisableBit, JointType, Model


# -- stage-group aliases --------------------------------------------------------------------------
def _position(m: Model, d: Data):
  _call("mjw_fwd_position", m, d)


def kinematics(m: Model, d: Data):
  """Forward kinematics (smooth.py:357-415): the position-stage launch."""
  _position(m, d)


def com_pos(m: Model, d: Data):
  """subtree_com, cinert, cdof (smooth.py:463-632): the position-stage launch."""
  _position(m, d)


def camlight(m: Model, d: Data):
  """Camera / light frames (smooth.py:635-803): the position-stage launch."""
  _position(m, d)


def flex(m: Model, d: Data):
  """Flex vertex positions and edge lengths / Jacobians (smooth.py:419-460): the position-stage launch."""
  _position(m, d)


def tendon(m: Model, d: Data):
  """Tendon lengths and Jacobians (smooth.py:3627-3700): the position-stage launch."""
  _position(m, d)


def crb(m: Model, d: Data):
  """Composite rigid-body inertia and qM (smooth.py:806-912): the position-stage launch."""
  _position(m, d)


def collision(m: Model, d: Data):
  """Broadphase + narrowphase into d.contact (collision_driver.py:757-789), with the contactfilter callback
  after it: the position-stage launch (fwd_position)."""
  fwd_position(m, d)


def make_constraint(m: Model, d: Data):
  """Constraint rows d.efc (constraint.py:2718-2779): the position-stage launch, whose rows come from the
  contacts it collides; after a caller edited d.contact, `mjw_contact_rows` rebuilds them from the pool."""
  _position(m, d)


def transmission(m: Model, d: Data):
  """Actuator lengths and moments (smooth.py:2605-2700): the position-stage launch."""
  _position(m, d)


def com_vel(m: Model, d: Data):
  """cvel, cdof_dot (smooth.py:1935-2038): the velocity-stage launch."""
  _call("mjw_fwd_velocity", m, d)


def passive(m: Model, d: Data):
  """qfrc_spring / damper / passive (passive.py:535-563): the velocity-stage launch (then the passive
  callback, as fwd_velocity)."""
  fwd_velocity(m, d)


def rne(m: Model, d: Data, flg_acc: bool = False):
  """qfrc_bias = RNE with zero acceleration (smooth.py:1276-1300, flg_acc = False): the velocity-stage
  launch.  flg_acc = True (the inverse-dynamics use, out of this build's scope) is refused."""
  if flg_acc:
    raise NotImplementedError("rne(flg_acc=True) (inverse dynamics) is not part of this build")
  _call("mjw_fwd_velocity", m, d)


def factor_m(m: Model, d: Data):
  """qLD = factor(qM) (smooth.py:1104-1112): the acceleration-stage launch (dense: Cholesky L, row-major
  nv x nv; sparse: L'DL on the ancestor rows, mj_factorM order)."""
  _call("mjw_fwd_acceleration", m, d)


def rne_postconstraint(m: Model, d: Data):
  """cacc, cfrc_int, cfrc_ext after the solver (smooth.py:1501-1600): the sensor kernel's acceleration
  stage (it also evaluates the acceleration sensors)."""
  _sensor(m, d, 4)


# -- support functions on caller arrays -------------------------------------------------------------
def _per_world(t: torch.Tensor, nworld: int, *shape) -> torch.Tensor:
  """A batched model field (leading dim 1 or nworld) as one row per world: types.py's `*` fields are read
  at worldid % nb."""
  t = t.reshape((-1,) + shape)
  return t[torch.arange(nworld, device=t.device) % t.shape[0]]


def _path_mask(m: Model) -> torch.Tensor:
  """(nbody, nbody) bool, [b, a]: body a lies on the path from b up to (not including) the world body."""
  mask = getattr(m, "_path_mask", None)
  if mask is None:
    par = m.body_parentid.cpu().numpy()
    nb = len(par)
    out = np.zeros((nb, nb), dtype=bool)
    for b in range(nb):
      p = b
      while p != 0:
        out[b, p] = True
        p = par[p]
    mask = torch.as_tensor(out, device=m.body_parentid.device)
    m._path_mask = mask
  return mask


def _cdof(m: Model, d: Data):
  c = d.cdof.reshape(d.nworld, m.nv, 6)
  return c[..., :3], c[..., 3:]  # angular (spatial top), linear (spatial bottom)


def jac(m: Model, d: Data, jacp: Optional[torch.Tensor], jacr: Optional[torch.Tensor], point: torch.Tensor, body: torch.Tensor):
  """Translational / rotational Jacobian of a point on a body, per world (support.py:397-503): dof i
  contributes when its body is on the path from `body` to the root (or is the world body), with
  jacp = cdof_lin + cdof_ang x (point - subtree_com[rootid[body]]) and jacr = cdof_ang.
  point: (nworld, 3); body: (nworld,) int; jacp / jacr: (nworld, 3, nv) outputs, either may be None."""
  body = body.to(torch.long).reshape(-1)
  ang, lin = _cdof(m, d)
  dof_body = m.dof_bodyid.to(torch.long)
  in_tree = (dof_body == 0).unsqueeze(0) | _path_mask(m)[body][:, dof_body]  # (nworld, nv)
  root = m.body_rootid.to(torch.long)[body]
  sc = d.subtree_com.reshape(d.nworld, m.nbody, 3)
  offset = point.reshape(-1, 3) - sc[torch.arange(d.nworld, device=sc.device), root]
  w = in_tree.to(ang.dtype).unsqueeze(-1)
  if jacp is not None:
    jp = (lin + torch.cross(ang, offset.unsqueeze(1).expand_as(ang), dim=-1)) * w
    jacp[:] = jp.transpose(1, 2)
  if jacr is not None:
    jacr[:] = (ang * w).transpose(1, 2)


def xfrc_accumulate(m: Model, d: Data, qfrc: torch.Tensor):
  """qfrc += J' xfrc_applied over every body (support.py:175-237 apply_ft): the body's force (xfrc[:3]) acts
  at xipos, its torque (xfrc[3:]) on the rotational Jacobian; dof i sees the bodies of its body's subtree."""
  ang, lin = _cdof(m, d)
  ft = d.xfrc_applied.reshape(d.nworld, m.nbody, 6)
  f, t = ft[..., :3], ft[..., 3:]
  sc = d.subtree_com.reshape(d.nworld, m.nbody, 3)
  off = d.xipos.reshape(d.nworld, m.nbody, 3) - sc[:, m.body_rootid.to(torch.long)]
  mask = _path_mask(m)[:, m.dof_bodyid.to(torch.long)].to(ang.dtype)  # (nbody, nv): dof's body on b's path
  # lin . f + ang . t + (ang x off) . f  =  lin . f + ang . (t + off x f)
  tq = t + torch.cross(off, f, dim=-1)
  qfrc += torch.einsum("wik,wbk,bi->wi", lin, f, mask) + torch.einsum("wik,wbk,bi->wi", ang, tq, mask)


def solve_m(m: Model, d: Data, x: torch.Tensor, y: torch.Tensor):
  """x = M^-1 y with the factor in d.qLD (smooth.py:2848-2858).  Dense: qLD holds the Cholesky factor L
  (M = L L'); sparse: L'DL on the ancestor rows (the sparse path's solve_trees order,
  smooth.py:2813-2846)."""
  nv = m.nv
  if not m.is_sparse:
    L = torch.tril(d.qLD.reshape(d.nworld, nv, nv))
    x[:] = torch.cholesky_solve(y.reshape(d.nworld, nv, 1), L).reshape(d.nworld, nv)
    return
  LD = d.qLD.reshape(d.nworld, -1)
  rowadr = m.M_rowadr.cpu().numpy()
  rownnz = m.M_rownnz.cpu().numpy()
  colind = m.M_colind.cpu().numpy()
  v = y.reshape(d.nworld, nv).clone()
  for k in range(nv - 1, -1, -1):
    a, n = int(rowadr[k]), int(rownnz[k])
    if n > 1:
      cols = torch.as_tensor(colind[a : a + n - 1], device=v.device, dtype=torch.long)
      v[:, cols] -= LD[:, a : a + n - 1] * v[:, k : k + 1]
  diag = torch.as_tensor(rowadr + rownnz - 1, device=v.device, dtype=torch.long)
  v /= LD[:, diag]
  for k in range(nv):
    a, n = int(rowadr[k]), int(rownnz[k])
    if n > 1:
      cols = torch.as_tensor(colind[a : a + n - 1], device=v.device, dtype=torch.long)
      v[:, k] -= (LD[:, a : a + n - 1] * v[:, cols]).sum(dim=1)
  x[:] = v


def subtree_vel(m: Model, d: Data):
  """subtree_linvel and subtree_angmom (smooth.py:2932-3083), stored on d as (nworld, nbody, 3) tensors and
  returned: each body's COM velocity and spin momentum, then linear momenta summed up the tree (deepest
  bodies first; DFS pre-order puts every descendant after its ancestors) and divided by the subtree mass,
  then angular momenta about the subtree COMs summed up the tree."""
  nw, nb = d.nworld, m.nbody
  mass = _per_world(m.body_mass, nw, nb)
  stm = _per_world(m.body_subtreemass, nw, nb)
  inertia = _per_world(m.body_inertia, nw, nb, 3)
  cvel = d.cvel.reshape(nw, nb, 6)
  xipos = d.xipos.reshape(nw, nb, 3)
  ximat = d.ximat.reshape(nw, nb, 3, 3)
  sc = d.subtree_com.reshape(nw, nb, 3)
  ang = cvel[..., :3]
  lin = cvel[..., 3:] - torch.cross(xipos - sc[:, m.body_rootid.to(torch.long)], ang, dim=-1)  # :2960
  linvel = mass.unsqueeze(-1) * lin
  dv = torch.einsum("wbji,wbj->wbi", ximat, ang) * inertia  # ximat' ang, scaled by the principal inertia
  angmom = torch.einsum("wbij,wbj->wbi", ximat, dv)
  par = m.body_parentid.cpu().numpy()
  for b in range(nb - 1, -1, -1):  # _linear_momentum (:2972-2988)
    if b:
      linvel[:, par[b]] += linvel[:, b]
    linvel[:, b] /= torch.clamp(stm[:, b : b + 1], min=1e-15)
  for b in range(nb - 1, 0, -1):  # _angular_momentum (:2992-3041)
    p = par[b]
    angmom[:, b] += torch.cross(xipos[:, b] - sc[:, b], (lin[:, b] - linvel[:, b]) * mass[:, b : b + 1], dim=-1)
    angmom[:, p] += angmom[:, b]
    angmom[:, p] += torch.cross(sc[:, b] - sc[:, p], (linvel[:, b] - linvel[:, p]) * stm[:, b : b + 1], dim=-1)
  d.subtree_linvel = linvel
  d.subtree_angmom = angmom
  return linvel, angmom


def _quat_sub(qa: torch.Tensor, qb: torch.Tensor) -> torch.Tensor:
  """math.py:162-185: qb * quat(res) = qa, as a 3D rotation vector."""
  w1, v1 = qb[..., :1], -qb[..., 1:]
  w2, v2 = qa[..., :1], qa[..., 1:]
  w = w1 * w2 - (v1 * v2).sum(-1, keepdim=True)
  v = w1 * v2 + w2 * v1 + torch.cross(v1, v2, dim=-1)
  s = torch.linalg.norm(v, dim=-1, keepdim=True)
  speed = 2.0 * torch.atan2(s, w)
  speed = torch.where(speed > np.pi, speed - 2.0 * np.pi, speed)
  return torch.where(s > 0, v * speed / torch.where(s > 0, s, torch.ones_like(s)), torch.zeros_like(v))


def energy_pos(m: Model, d: Data):
  """d.energy[:, 0] = potential energy (sensor.py:2854-2890): gravity -sum mass g . xipos over the bodies
  and joint / tendon springs 0.5 k dif^2 (free joints: translation and rotation, ball joints: rotation)."""
  nw, nb = d.nworld, m.nbody
  e = torch.zeros(nw, dtype=d.energy.dtype, device=d.energy.device)
  if not (m.opt.disableflags & DisableBit.GRAVITY):
    g = _per_world(m.opt.gravity, nw, 3)
    mass = _per_world(m.body_mass, nw, nb)
    xipos = d.xipos.reshape(nw, nb, 3)
    e -= (mass[:, 1:] * (xipos[:, 1:] * g[:, None, :]).sum(-1)).sum(dim=1)
  if not (m.opt.disableflags & DisableBit.SPRING):
    # batched (*) stiffness, spring reference and tendon spring lengths are read per world at worldid % nb,
    # as sensor.py's _energy_pos_* kernels do; a joint / tendon counts when any world's stiffness is non-zero
    stiff = _per_world(m.jnt_stiffness, nw, m.njnt)
    jt = m.jnt_type.cpu().numpy()
    qa_all = m.jnt_qposadr.cpu().numpy()
    qs = _per_world(m.qpos_spring, nw, m.nq)
    qpos = d.qpos.reshape(nw, m.nq)
    for j in np.nonzero((m.jnt_stiffness.reshape(-1, m.njnt) != 0).any(dim=0).cpu().numpy())[0]:
      k, qa = stiff[:, j], int(qa_all[j])
      if jt[j] == JointType.FREE:
        d0 = qpos[:, qa : qa + 3] - qs[:, qa : qa + 3]
        q1 = torch.nn.functional.normalize(qpos[:, qa + 3 : qa + 7], dim=-1)
        d1 = _quat_sub(q1, qs[:, qa + 3 : qa + 7])
        e += 0.5 * k * ((d0 * d0).sum(-1) + (d1 * d1).sum(-1))
      elif jt[j] == JointType.BALL:
        q = torch.nn.functional.normalize(qpos[:, qa : qa + 4], dim=-1)
        dq = _quat_sub(q, qs[:, qa : qa + 4])
        e += 0.5 * k * (dq * dq).sum(-1)
      else:
        dq = qpos[:, qa] - qs[:, qa]
        e += 0.5 * k * dq * dq
    nten = getattr(m, "ntendon", 0)
    if nten:
      tstiff = _per_world(m.tendon_stiffness, nw, nten)
      tls = _per_world(m.tendon_lengthspring, nw, nten, 2)
      for t in np.nonzero((m.tendon_stiffness.reshape(-1, nten) != 0).any(dim=0).cpu().numpy())[0]:
        k, lo, hi = tstiff[:, t], tls[:, t, 0], tls[:, t, 1]
        length = d.ten_length.reshape(nw, nten)[:, t]
        disp = torch.where(length > hi, hi - length, torch.where(length < lo, lo - length, torch.zeros_like(length)))
        e += 0.5 * k * disp * disp
  d.energy.reshape(nw, 2)[:, 0] = e


def energy_vel(m: Model, d: Data):
  """d.energy[:, 1] = kinetic energy 0.5 qvel' M qvel (sensor.py:2922-2940, mul_m on qM)."""
  from .support import mul_m

  mv = torch.zeros_like(d.qvel)
  mul_m(m, d, mv, d.qvel)
  d.energy.reshape(d.nworld, 2)[:, 1] = 0.5 * (d.qvel * mv).sum(dim=1)


def set_const_fixed(m: Model, d: Data):
  """The qpos0-independent derived constants (io.py:2197-2219): body_subtreemass = the body's mass plus
  its descendants', per model row (a body_mass batched per world gives a per-world body_subtreemass, which
  the kernels then read at worldid % nb).  The rest of the set_const family (qpos0-dependent invweights,
  acc0, camera / light references) is derived by put_model and not recomputed on the device."""
  nb = m.nbody
  mass = m.body_mass.reshape(-1, nb)
  sub = mass.clone()
  par = m.body_parentid.cpu().numpy()
  for b in range(nb - 1, 0, -1):  # DFS pre-order: descendants follow their ancestors
    sub[:, par[b]] += sub[:, b]
  m.body_subtreemass = sub.to(m.body_subtreemass.dtype).contiguous()


def set_const_0(m: Model, d: Data):
  """The qpos0-dependent derived constants (io.py:2222-2407) on the device, per world: the position stage at
  qpos0 (then qpos is restored), then from qM and its inverse stat.meaninertia (trace / nv),
  dof_invweight0 (diag M^-1, averaged per free-joint translation / rotation and per ball joint),
  body_invweight0 (mean translational / rotational diagonal of J M^-1 J' at the body COM; zero for the world
  and static bodies), tendon_invweight0 (J M^-1 J') and actuator_acc0 (||M^-1 moment||, joint and tendon
  transmissions), the camera / light references -- the same definitions mjcf.py's compiler applies on
  the host.  Dense models; the dampratio resolution keeps put_model's values."""
  if m.is_sparse:
    raise NotImplementedError("set_const_0 on sparse models is not part of this build")
  nw, nv, nb = d.nworld, m.nv, m.nbody
  saved = d.qpos.clone()
  d.qpos[:] = _per_world(m.qpos0, nw, m.nq)
  _call("mjw_fwd_position", m, d)
  M = d.qM.reshape(nw, m.nv_pad, m.nv_pad)[:, :nv, :nv].double()
  Minv = torch.linalg.inv(M)
  f32 = m.dof_invweight0.dtype
  m.stat.meaninertia = (M.diagonal(dim1=1, dim2=2).sum(1) / max(nv, 1)).to(f32)
  diag = Minv.diagonal(dim1=1, dim2=2)
  jt, jda = m.jnt_type.cpu().numpy(), m.jnt_dofadr.cpu().numpy()
  inv = torch.zeros_like(diag)
  for i, j in enumerate(m.dof_jntid.cpu().numpy()):
    da = int(jda[j])
    if jt[j] == JointType.FREE:
      inv[:, i] = diag[:, da : da + 3].mean(1) if i < da + 3 else diag[:, da + 3 : da + 6].mean(1)
    elif jt[j] == JointType.BALL:
      inv[:, i] = diag[:, da : da + 3].mean(1)
    else:
      inv[:, i] = diag[:, i]
  m.dof_invweight0 = inv.to(f32)
  # body_invweight0 at the body COMs
  biw = torch.zeros(nw, nb, 2, dtype=torch.float64, device=M.device)
  weld = m.body_weldid.cpu().numpy()
  jacp = torch.zeros(nw, 3, nv, device=M.device)
  jacr = torch.zeros(nw, 3, nv, device=M.device)
  xipos = d.xipos.reshape(nw, nb, 3)
  for b in range(1, nb):
    if weld[b] == 0 or nv == 0:
      continue
    jac(m, d, jacp, jacr, xipos[:, b], torch.full((nw,), b, device=M.device))
    J = torch.cat([jacp, jacr], dim=1).double()
    A = J @ Minv @ J.transpose(1, 2)
    ad = A.diagonal(dim1=1, dim2=2)
    tr, rot = ad[:, :3].mean(1), ad[:, 3:].mean(1)
    tr2 = torch.where((tr < 1e-15) & (rot > 1e-15), rot, tr)
    rot2 = torch.where((rot < 1e-15) & (tr > 1e-15), tr, rot)
    biw[:, b, 0], biw[:, b, 1] = tr2, rot2
  m.body_invweight0 = biw.to(f32)
  # tendons: dense Jacobian rows from the sparse ten_J pattern
  nt = int(getattr(m, "ntendon", 0))
  tenJ = torch.zeros(nw, nt, nv, dtype=torch.float64, device=M.device)
  if nt:
    rownnz, rowadr, colind = (getattr(m, f).cpu().numpy() for f in ("ten_J_rownnz", "ten_J_rowadr", "ten_J_colind"))
    vals = d.ten_J.reshape(nw, -1).double()
    for t in range(nt):
      for k in range(int(rownnz[t])):
        tenJ[:, t, int(colind[rowadr[t] + k])] = vals[:, rowadr[t] + k]
    m.tendon_invweight0 = torch.einsum("wti,wij,wtj->wt", tenJ, Minv, tenJ).to(f32)
  # actuator_acc0
  if m.nu:
    gear = _per_world(m.actuator_gear, nw, m.nu, 6).double()
    trn, trnid = m.actuator_trntype.cpu().numpy(), m.actuator_trnid.reshape(-1, 2).cpu().numpy()
    vec = torch.zeros(nw, m.nu, nv, dtype=torch.float64, device=M.device)
    for a in range(m.nu):
      j = int(trnid[a, 0])
      if trn[a] == 3:  # TrnType.TENDON
        vec[:, a] = gear[:, a, :1] * tenJ[:, j]
        continue
      da = int(jda[j])
      if jt[j] == JointType.FREE:
        vec[:, a, da : da + 6] = gear[:, a]
      elif jt[j] == JointType.BALL:
        vec[:, a, da : da + 3] = gear[:, a, :3]
      else:
        vec[:, a, da] = gear[:, a, 0]
    m.actuator_acc0 = torch.linalg.norm(torch.einsum("wij,waj->wai", Minv, vec), dim=-1).to(f32)
  # camera / light references at qpos0 (io.py:2330-2345): the fixed-frame placement relative to the body
  # and to the target's (or own) subtree COM
  xpos = d.xpos.reshape(nw, nb, 3)
  xmat = d.xmat.reshape(nw, nb, 3, 3)
  sc = d.subtree_com.reshape(nw, nb, 3)
  if m.ncam:
    b = m.cam_bodyid.to(torch.long)
    tgt = m.cam_targetbodyid.to(torch.long)
    ref = torch.where(tgt >= 0, tgt, b)
    cpos = _per_world(m.cam_pos, nw, m.ncam, 3)
    cq = torch.nn.functional.normalize(_per_world(m.cam_quat, nw, m.ncam, 4), dim=-1)
    cx = xpos[:, b] + torch.einsum("wcij,wcj->wci", xmat[:, b], cpos)
    m.cam_pos0 = (cx - xpos[:, b]).to(f32)
    m.cam_poscom0 = (cx - sc[:, ref]).to(f32)
    m.cam_mat0 = torch.einsum("wcij,wcjk->wcik", xmat[:, b], _quat_to_mat(cq)).reshape(nw, m.ncam, 9).to(f32)
  if m.nlight:
    b = m.light_bodyid.to(torch.long)
    tgt = m.light_targetbodyid.to(torch.long)
    ref = torch.where(tgt >= 0, tgt, b)
    lx = xpos[:, b] + torch.einsum("wlij,wlj->wli", xmat[:, b], _per_world(m.light_pos, nw, m.nlight, 3))
    m.light_pos0 = (lx - xpos[:, b]).to(f32)
    m.light_poscom0 = (lx - sc[:, ref]).to(f32)
    m.light_dir0 = torch.einsum("wlij,wlj->wli", xmat[:, b], _per_world(m.light_dir, nw, m.nlight, 3)).to(f32)
  d.qpos[:] = saved


def _quat_to_mat(q: torch.Tensor) -> torch.Tensor:
  """math.py quat_to_mat for unit quaternions (..., 4) -> (..., 3, 3)."""
  w, x, y, z = q.unbind(-1)
  r = torch.stack([
    1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
    2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
    2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], dim=-1)
  return r.reshape(q.shape[:-1] + (3, 3))


def set_const(m: Model, d: Data):
  """set_const_fixed then set_const_0 (io.py:2410-2470)."""
  set_const_fixed(m, d)
  set_const_0(m, d)
