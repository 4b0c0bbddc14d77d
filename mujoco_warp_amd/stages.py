"""The reference's finer-grained stage and support functions.

`mujoco_warp` exposes every pipeline stage as its own function (mujoco_warp/__init__.py:26-112:
`kinematics`, `com_pos`, `crb`, `collision`, `make_constraint`, `rne`, ...).  The step fuses them into
one launch per stage group; on their own they run as follows:

* dense-path models (round 6): `kinematics`, `com_pos`, `camlight`, `tendon`, `crb`, `make_constraint`,
  `transmission`, `com_vel`, `passive` and `rne` each launch that one stage (`mjw_stage`, one wave per
  world): its inputs are the Data fields the earlier stages wrote -- a caller's edit of e.g. `d.xipos`
  before `com_pos` is what `com_pos` reads, as in the reference -- and only its own outputs are written;
* `collision` and `flex`, and every stage of sparse / flex models (the workgroup-per-world pipeline):
  the launch that contains the stage (`mjw_fwd_position` / `mjw_fwd_velocity`), which recomputes the
  stage's inputs from `qpos` / `qvel` and writes the group's other outputs along with it; so does
  `transmission` for models with BODY (adhesion) transmissions, which accumulate over the collision's
  contacts;
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
from . import types
from .types import Data, DisableBit, JointType, Model


# -- stages ---------------------------------------------------------------------------------------
def _position(m: Model, d: Data):
  _call("mjw_fwd_position", m, d)


# include/mjw_amd.h MJW_STAGE_*
STAGE_IDS = {"kinematics": 1, "com_pos": 2, "camlight": 3, "tendon": 4, "crb": 5, "make_constraint": 6, "transmission": 7,
             "com_vel": 8, "passive": 9, "rne": 10}


def _stage(name: str, m: Model, d: Data) -> bool:
  """Launch one stage (mjw_stage) on a dense-path model; False when the model needs the stage group's
  launch instead (sparse / flex models, BODY transmissions)."""
  if m.is_sparse or (name == "transmission" and int(m.nbodytrn) > 0):
    return False
  from . import _lib
  from .forward import _stream
  from .io import cdata, cmodel

  L = _lib.lib()
  _lib.check(L.mjw_stage(cmodel(m), cdata(d), STAGE_IDS[name], _stream(d)), f"mjw_stage({name})")
  return True


def kinematics(m: Model, d: Data):
  """Forward kinematics (smooth.py:357-415): body, joint, geom and site frames from qpos / mocap."""
  if not _stage("kinematics", m, d):
    _position(m, d)


def com_pos(m: Model, d: Data):
  """subtree_com, cinert, cdof (smooth.py:601-632) from the frames in d."""
  if not _stage("com_pos", m, d):
    _position(m, d)


def camlight(m: Model, d: Data):
  """Camera / light frames (smooth.py:635-803) from the frames and subtree_com in d."""
  if not _stage("camlight", m, d):
    _position(m, d)


def flex(m: Model, d: Data):
  """Flex vertex positions and edge lengths / Jacobians (smooth.py:419-460): the position-stage launch
  (flexes run on the sparse pipeline)."""
  _position(m, d)


def tendon(m: Model, d: Data):
  """Tendon lengths and Jacobians (smooth.py:3627-3700) from qpos and the frames in d."""
  if not _stage("tendon", m, d):
    _position(m, d)


def crb(m: Model, d: Data):
  """Composite rigid-body inertia and qM (smooth.py:888-912, tendon armature included) from cinert / cdof."""
  if not _stage("crb", m, d):
    _position(m, d)


def collision(m: Model, d: Data):
  """Broadphase + narrowphase into d.contact (collision_driver.py:757-789), with the contactfilter callback
  after it: the position-stage launch (fwd_position)."""
  fwd_position(m, d)


# -- collision sub-stages (mujoco_warp/__init__.py:33-35) ---------------------------------------------------
class CollisionContext(types._Container):
  """Broadphase output arrays (collision_core.py:345-357), each naconmax long: collision_pair (n, 2) int32
  type-ordered geom ids, collision_pairid (n, 2) int32 (explicit <pair> id or -1 / -2 excluded, collision-
  sensor id or -1), collision_worldid (n,) int32."""


def create_collision_context(naconmax: int, device=None) -> CollisionContext:
  """collision_core.py:359-365 (device: the Data's device when given as a Data, else cuda)."""
  if isinstance(device, Data):
    device = device.qpos.device
  dev = torch.device(device) if device is not None else torch.device("cuda")
  n = int(naconmax)
  return CollisionContext(
    collision_pair=torch.full((n, 2), -1, dtype=torch.int32, device=dev),
    collision_pairid=torch.full((n, 2), -1, dtype=torch.int32, device=dev),
    collision_worldid=torch.full((n,), -1, dtype=torch.int32, device=dev),
  )


def _ctx_ptrs(d: Data, ctx: CollisionContext):
  for name in ("collision_pair", "collision_pairid", "collision_worldid"):
    t = getattr(ctx, name)
    if t.dtype != torch.int32 or not t.is_contiguous() or t.shape[0] < d.naconmax:
      raise ValueError(f"CollisionContext.{name}: int32, contiguous, at least naconmax = {d.naconmax} rows")
  return ctx.collision_pair.data_ptr(), ctx.collision_pairid.data_ptr(), ctx.collision_worldid.data_ptr()


def nxn_broadphase(m: Model, d: Data, ctx: CollisionContext):
  """collision_driver.py:697-731: the filtered NXN pairs that pass opt.broadphase_filter (plane / sphere /
  AABB / OBB, :274-321) at the current d.geom_xpos / d.geom_xmat, appended to `ctx` with d.ncollision
  counting them (the caller zeroes it, as `collision` does); pairs with a collision sensor always pass.
  One thread per (world, pair) (mjw_nxn_broadphase); the order of the candidates is the atomics' order."""
  from . import _lib
  from .io import cdata, cmodel
  from .forward import _stream

  L = _lib.lib()
  pp, pi, pw = _ctx_ptrs(d, ctx)
  _lib.check(L.mjw_nxn_broadphase(cmodel(m), cdata(d), pp, pi, pw, _stream(d)), "mjw_nxn_broadphase")


def sap_broadphase(m: Model, d: Data, ctx: CollisionContext):
  """collision_driver.py:554-643 sweep-and-prune: per world the geoms' bounding spheres (rbound + margin,
  planes unbounded) projected on the reference's fixed direction and sorted in LDS, each sorted geom's
  candidates up to the first one past its overlap (_sap_range :421-441), those that are NXN pairs through the
  broadphase filter (or with a collision-sensor id) appended to `ctx` as nxn_broadphase does, d.ncollision
  counting them.  One workgroup per world (mjw_sap_broadphase, ngeom <= 4096)."""
  from . import _lib
  from .io import cdata, cmodel
  from .forward import _stream

  L = _lib.lib()
  pp, pi, pw = _ctx_ptrs(d, ctx)
  _lib.check(L.mjw_sap_broadphase(cmodel(m), cdata(d), pp, pi, pw, _stream(d)), "mjw_sap_broadphase")


# the PRIMITIVE entries of collision_driver.py:43-77 (type-ordered pairs)
PRIMITIVE_PAIRS = (
  (types.GeomType.PLANE, types.GeomType.SPHERE), (types.GeomType.PLANE, types.GeomType.CAPSULE),
  (types.GeomType.PLANE, types.GeomType.ELLIPSOID), (types.GeomType.PLANE, types.GeomType.CYLINDER),
  (types.GeomType.PLANE, types.GeomType.BOX), (types.GeomType.PLANE, types.GeomType.MESH),
  (types.GeomType.SPHERE, types.GeomType.SPHERE), (types.GeomType.SPHERE, types.GeomType.CAPSULE),
  (types.GeomType.SPHERE, types.GeomType.CYLINDER), (types.GeomType.SPHERE, types.GeomType.BOX),
  (types.GeomType.CAPSULE, types.GeomType.CAPSULE), (types.GeomType.CAPSULE, types.GeomType.BOX),
)


def primitive_narrowphase(m: Model, d: Data, ctx: CollisionContext, collision_table=None):
  """collision_primitive.py:1461-1549: contacts of the broadphase candidates whose (type-ordered) geom types
  are in `collision_table` (default: every PRIMITIVE pair), appended to d.contact at d.nacon with
  write_contact's rules (collision_core.py:160-232: inactive points are kept only for collision sensors;
  type = CONSTRAINT | SENSOR bits; efc_address -1 until make_constraint).  One thread per candidate
  (mjw_primitive_narrowphase), the fused path's geometry routines."""
  from . import _lib
  from .io import cdata, cmodel
  from .forward import _stream

  table = PRIMITIVE_PAIRS if collision_table is None else collision_table
  mask = 0
  for t1, t2 in table:
    a, b = sorted((int(t1), int(t2)))
    if (a, b) not in {(int(x), int(y)) for x, y in PRIMITIVE_PAIRS}:
      raise NotImplementedError(f"primitive_narrowphase: ({types.GeomType(a).name}, {types.GeomType(b).name}) is not a primitive pair")
    mask |= 1 << (8 * a + b)
  L = _lib.lib()
  pp, pi, pw = _ctx_ptrs(d, ctx)
  _lib.check(L.mjw_primitive_narrowphase(cmodel(m), cdata(d), pp, pi, pw, mask, _stream(d)), "mjw_primitive_narrowphase")


def make_constraint(m: Model, d: Data):
  """Constraint rows d.efc (constraint.py:2718-2779) from the contacts in d.contact and the frames in d
  (dense path; the sparse path reruns its position launch)."""
  if not _stage("make_constraint", m, d):
    _position(m, d)


def transmission(m: Model, d: Data):
  """Actuator lengths and moments (smooth.py:2605-2700) from the frames in d (BODY transmissions: the
  position-stage launch, their moments sum over its contacts)."""
  if not _stage("transmission", m, d):
    _position(m, d)


def com_vel(m: Model, d: Data):
  """cvel, cdof_dot (smooth.py:1935-2038) and actuator_velocity from qvel and the frames in d."""
  if not _stage("com_vel", m, d):
    _call("mjw_fwd_velocity", m, d)


def passive(m: Model, d: Data):
  """qfrc_spring / damper / gravcomp / fluid / passive (passive.py:535-563) from the state in d, then the
  passive callback (as fwd_velocity calls it)."""
  if not _stage("passive", m, d):
    fwd_velocity(m, d)
    return
  if m.callback.passive is not None:
    m.callback.passive(m, d)


def rne(m: Model, d: Data, flg_acc: bool = False):
  """qfrc_bias = RNE with zero acceleration (smooth.py:1276-1300, flg_acc = False) from cvel / cdof_dot
  in d.  flg_acc = True (the inverse-dynamics use, out of this build's scope) is refused."""
  if flg_acc:
    raise NotImplementedError("rne(flg_acc=True) (inverse dynamics) is not part of this build")
  if not _stage("rne", m, d):
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
  the host.  Sparse models expand their ancestor-row qM (M_rowadr / M_rownnz / M_colind) to the dense
  symmetric matrix first.  The dampratio resolution keeps put_model's values."""
  nw, nv, nb = d.nworld, m.nv, m.nbody
  saved = d.qpos.clone()
  # the position launch also runs collision and make_constraint, which the reference's set_const_0 does not
  # (io.py:2245-2253 runs the smooth stages only): the contact pool and the constraint rows are restored
  kept = {k: getattr(d, k).clone() for k in ("nacon", "ncollision", "ne", "nf", "nl", "nefc") if torch.is_tensor(getattr(d, k, None))}
  kept_sub = {(g, k): v.clone() for g in ("contact", "efc") for k, v in vars(getattr(d, g)).items() if torch.is_tensor(v)}
  d.qpos[:] = _per_world(m.qpos0, nw, m.nq)
  _call("mjw_fwd_position", m, d)
  if int(getattr(m, "ntendon", 0)):  # io.py:2263 tendon_length0 from ten_length at qpos0
    m.tendon_length0 = d.ten_length.reshape(nw, m.ntendon).to(m.tendon_length0.dtype).clone()
  if m.is_sparse:
    rownnz = m.M_rownnz.reshape(-1).to(torch.long)
    rows = torch.repeat_interleave(torch.arange(nv, device=rownnz.device), rownnz)
    adr = torch.cat([torch.arange(int(a), int(a) + int(n)) for a, n in zip(m.M_rowadr.reshape(-1).tolist(), rownnz.tolist())]).to(rows.device)
    cols = m.M_colind.reshape(-1).to(torch.long)[adr]
    vals = d.qM.reshape(nw, -1)[:, adr].double()
    M = torch.zeros(nw, nv, nv, dtype=torch.float64, device=d.qM.device)
    M[:, cols, rows] = vals
    M[:, rows, cols] = vals
  else:
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
  for k, v in kept.items():
    getattr(d, k).copy_(v)
  for (g, k), v in kept_sub.items():
    getattr(getattr(d, g), k).copy_(v)


def _quat_to_mat(q: torch.Tensor) -> torch.Tensor:
  """math.py quat_to_mat for unit quaternions (..., 4) -> (..., 3, 3)."""
  w, x, y, z = q.unbind(-1)
  r = torch.stack([
    1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
    2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
    2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], dim=-1)
  return r.reshape(q.shape[:-1] + (3, 3))


def set_length_range(m: Model, d: Data, index: int = -1):
  """io.py:2465-2495 (with _set_length_range :2158-2194): the actuator length ranges from the limits of joint
  and tendon transmissions scaled by gear[0] (swapped for a negative gear); every other actuator gets (0, 0),
  as the reference writes them.  One row per world (actuator_gear / jnt_range / tendon_range are read at
  worldid % nb).  `index` is accepted for API parity and, as in the reference, does not restrict the update."""
  del index
  nu, nw = m.nu, d.nworld
  if nu == 0:
    return
  dev = m.actuator_gear.device
  trn = m.actuator_trntype.long()
  id0 = m.actuator_trnid.reshape(nu, 2)[:, 0].long()
  gear0 = _per_world(m.actuator_gear, nw, nu, 6)[:, :, 0].double()
  lr = torch.zeros(nw, nu, 2, dtype=torch.float64, device=dev)
  joint = (trn == int(types.TrnType.JOINT)) | (trn == int(types.TrnType.JOINTINPARENT))
  if m.njnt:
    jl = m.jnt_limited.long()[id0.clamp(0, m.njnt - 1)] != 0
    rng = _per_world(m.jnt_range, nw, m.njnt, 2).double()[:, id0.clamp(0, m.njnt - 1)]
    sel = (joint & jl)[None, :, None].expand(nw, nu, 2)
    lr = torch.where(sel, rng * gear0[:, :, None], lr)
  nten = int(getattr(m, "ntendon", 0))
  if nten:
    ten = trn == int(types.TrnType.TENDON)
    tl = m.tendon_limited.long()[id0.clamp(0, nten - 1)] != 0
    rng = _per_world(m.tendon_range, nw, nten, 2).double()[:, id0.clamp(0, nten - 1)]
    sel = (ten & tl)[None, :, None].expand(nw, nu, 2)
    lr = torch.where(sel, rng * gear0[:, :, None], lr)
  neg = (gear0 <= 0.0)[:, :, None].expand(nw, nu, 2)
  lr = torch.where(neg, lr.flip(-1), lr)  # gear <= 0: (rng[1] gear, rng[0] gear)
  m.actuator_lengthrange = lr.to(m.actuator_lengthrange.dtype).contiguous()


def deriv_smooth_vel(m: Model, d: Data, out: torch.Tensor):
  """derivative.py:321-416: out = qM - dt qDeriv, the derivative of the smooth forces with respect to qvel on
  the qM pattern: qDeriv = sum_a vel_a m_a m_a' (_qderiv_actuator_passive_vel: affine gain / bias slope, with
  the activation or control and the force-range cut) - diag(dof_damping) - sum_t damping_t J_t' J_t.  `out` has
  qM's shape: (nworld, nv_pad, nv_pad) dense, (nworld, nM) sparse.  The device implicitfast integrator forms
  the same matrix inside its Euler launch; this is the reference's stand-alone entry point."""
  nw, nv, nu = d.nworld, m.nv, m.nu
  dev = d.qM.device
  fl = int(m.opt.disableflags)
  dt = _per_world(m.opt.timestep, nw, 1)[:, 0].double()
  qd = torch.zeros(nw, nv, nv, dtype=torch.float64, device=dev)
  if nu and not (fl & int(DisableBit.ACTUATION)):
    gt, bt, dyn = m.actuator_gaintype.long(), m.actuator_biastype.long(), m.actuator_dyntype.long()
    gain = torch.where(gt == int(types.GainType.AFFINE), _per_world(m.actuator_gainprm, nw, nu, 10)[:, :, 2].double(), 0.0)
    bias = torch.where(bt == int(types.BiasType.AFFINE), _per_world(m.actuator_biasprm, nw, nu, 10)[:, :, 2].double(), 0.0)
    force = d.actuator_force.reshape(nw, nu).double()
    frng = _per_world(m.actuator_forcerange, nw, nu, 2).double()
    clamped = (m.actuator_forcelimited.bool())[None] & ((force <= frng[:, :, 0]) | (force >= frng[:, :, 1]))
    vel = bias.clone()
    na = int(m.na)
    if na:
      adr = (m.actuator_actadr.long() + m.actuator_actnum.long() - 1).clamp(0, na - 1)
      act = d.act.reshape(nw, na).double()[:, adr]
      act_dot = d.act_dot.reshape(nw, na).double()[:, adr]
      tau = _per_world(m.actuator_dynprm, nw, nu, 10)[:, :, 0].double().clamp_min(1e-15)
      nxt = torch.where(dyn == int(types.DynType.FILTEREXACT), act + act_dot * tau * (1 - torch.exp(-dt[:, None] / tau)), act + act_dot * dt[:, None])
      nxt = torch.where(dyn == int(types.DynType.USER), act, nxt)
      arng = _per_world(m.actuator_actrange, nw, nu, 2).double()
      nxt = torch.where(m.actuator_actlimited.bool()[None], torch.minimum(torch.maximum(nxt, arng[:, :, 0]), arng[:, :, 1]), nxt)
      act_use = torch.where(m.actuator_actearly.bool()[None], nxt, act)
    else:
      act_use = torch.zeros(nw, nu, dtype=torch.float64, device=dev)
    ctrl = d.ctrl.reshape(nw, nu).double()
    vel = vel + torch.where(dyn != int(types.DynType.NONE), gain * act_use, gain * ctrl)
    vel = torch.where(((gain == 0) & (bias == 0)) | clamped, 0.0, vel)
    mom = _moment_dense(m, d)  # (nw, nu, nv)
    qd += torch.einsum("wa,wai,waj->wij", vel, mom, mom)
  if not (fl & int(DisableBit.DAMPER)):
    qd -= torch.diag_embed(_per_world(m.dof_damping, nw, nv).double())
    nten = int(getattr(m, "ntendon", 0))
    if nten:
      J = _ten_J_dense(m, d)  # (nw, nten, nv)
      qd -= torch.einsum("wt,wti,wtj->wij", _per_world(m.tendon_damping, nw, nten).double(), J, J)
  res = _dense_qM(m, d).double() - dt[:, None, None] * qd
  # the reference fills the qM pattern only (qM_fullm_i / j: a dof and its ancestors)
  pat = _qM_pattern(m).to(dev)
  res = torch.where(pat[None], res, 0.0)
  if m.is_sparse:
    rows, cols = _sparse_index(m)
    out.reshape(nw, -1)[:, : m.nM] = res[:, rows, cols].to(out.dtype)
  else:
    out.zero_()
    out[:, :nv, :nv] = res.to(out.dtype)


def _moment_dense(m: Model, d: Data) -> torch.Tensor:
  """actuator_moment as (nworld, nu, nv) fp64 from its per-world sparse rows (moment_rownnz / rowadr / colind)."""
  nw, nu, nv = d.nworld, m.nu, m.nv
  nJ = int(m.nJmom)
  rnz = d.moment_rownnz.reshape(nw, nu).long()
  radr = d.moment_rowadr.reshape(nw, nu).long()
  col = d.moment_colind.reshape(nw, -1)[:, :nJ].long()
  val = d.actuator_moment.reshape(nw, -1)[:, :nJ].double()
  k = torch.arange(nJ, device=val.device)
  # actuator of slot k: rowadr <= k < rowadr + rownnz
  owner = ((k[None, None, :] >= radr[:, :, None]) & (k[None, None, :] < (radr + rnz)[:, :, None]))  # (nw, nu, nJ)
  out = torch.zeros(nw, nu, nv, dtype=torch.float64, device=val.device)
  out.scatter_add_(2, col[:, None, :].expand(nw, nu, nJ), torch.where(owner, val[:, None, :], 0.0))
  return out


def _ten_J_dense(m: Model, d: Data) -> torch.Tensor:
  """ten_J as (nworld, ntendon, nv) fp64 (the model's fixed row pattern ten_J_rownnz / rowadr / colind)."""
  nw, nten, nv = d.nworld, int(m.ntendon), m.nv
  nJ = int(m.nJten)
  rnz, radr, col = m.ten_J_rownnz.long(), m.ten_J_rowadr.long(), m.ten_J_colind.long()
  val = d.ten_J.reshape(nw, -1)[:, :nJ].double()
  out = torch.zeros(nw, nten, nv, dtype=torch.float64, device=val.device)
  for t in range(nten):
    a, n = int(radr[t]), int(rnz[t])
    out[:, t].index_add_(1, col[a:a + n], val[:, a:a + n])
  return out


def _qM_pattern(m: Model) -> torch.Tensor:
  """(nv, nv) bool: i, j in the same dof chain (the ancestor pattern qM stores, both triangles)."""
  nv = m.nv
  par = m.dof_parentid.cpu().numpy()
  pat = np.zeros((nv, nv), dtype=bool)
  for i in range(nv):
    j = i
    while j >= 0:
      pat[i, j] = pat[j, i] = True
      j = par[j]
  return torch.as_tensor(pat)


def _sparse_index(m: Model):
  """Row / column of every entry of the sparse qM layout (M_rowadr / M_colind: ancestors ascending, then the
  diagonal)."""
  rowadr = m.M_rowadr.cpu().numpy()
  rownnz = m.M_rownnz.cpu().numpy()
  colind = m.M_colind.cpu().numpy()
  rows = np.zeros(m.nM, dtype=np.int64)
  for i in range(m.nv):
    rows[rowadr[i]:rowadr[i] + rownnz[i]] = i
  return torch.as_tensor(rows), torch.as_tensor(colind.astype(np.int64))


def _dense_qM(m: Model, d: Data) -> torch.Tensor:
  """qM of every world as (nworld, nv, nv), from either layout."""
  nw, nv = d.nworld, m.nv
  if not m.is_sparse:
    return d.qM[:, :nv, :nv]
  rows, cols = _sparse_index(m)
  q = d.qM.reshape(nw, -1)[:, : m.nM]
  full = torch.zeros(nw, nv, nv, dtype=q.dtype, device=q.device)
  full[:, rows.to(q.device), cols.to(q.device)] = q
  full[:, cols.to(q.device), rows.to(q.device)] = q
  return full


def set_const(m: Model, d: Data):
  """set_const_fixed then set_const_0 (io.py:2410-2470)."""
  set_const_fixed(m, d)
  set_const_0(m, d)
