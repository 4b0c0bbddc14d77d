"""Host I/O: put_model / put_data / make_data / get_data_into / reset_data / override_model.

Mirrors mujoco_warp/_src/io.py: `put_model` (io.py:77-647) turns a compiled
model (this package's `mjcf.MjModel`, or a real `mujoco.MjModel` when that
package is importable) into device tensors plus the derived index arrays the
kernels need; `put_data` (io.py:1016-1240) tiles one host state over `nworld`
worlds; array shapes follow `types.Data` (types.py:1702-1896).  All device
memory is owned by torch tensors; the C ABI only receives their pointers.
"""

from __future__ import annotations

import ctypes
import dataclasses
from typing import Optional, Sequence

import os

import numpy as np
import torch

from . import _lib
from . import types
from .types import BroadphaseFilter, DisableBit, EnableBit, JointType

# reference io.py:650-661
def _round_up(x, k):
  return ((x + k - 1) // k) * k


def _padded_sizes(nv: int, njmax: int, is_sparse: bool):
  tile = types.TILE_SIZE_JTDAJ_SPARSE if is_sparse else types.TILE_SIZE_JTDAJ_DENSE
  njmax_pad = _round_up(njmax, tile)
  nv_pad = _round_up(nv, tile) if (is_sparse or nv > 32) else _round_up(nv, 4)
  return njmax_pad, nv_pad


def _muscle_mask(mjm):
  """Actuators with a muscle gain, bias or activation (forward.py:671-727)."""
  if not mjm.nu:
    return np.zeros(0, dtype=bool)
  return ((np.asarray(mjm.actuator_dyntype) == types.DynType.MUSCLE) | (np.asarray(mjm.actuator_gaintype) == types.GainType.MUSCLE)
          | (np.asarray(mjm.actuator_biastype) == types.BiasType.MUSCLE))


def is_sparse(mjm) -> bool:
  """io.py:67-74."""
  if mjm.opt.jacobian == types.JacobianType.AUTO:
    return mjm.nv > 32
  return mjm.opt.jacobian == types.JacobianType.SPARSE


def _device(device=None):
  if device is not None:
    return torch.device(device)
  return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")


def _f32(a, device):
  return torch.as_tensor(np.ascontiguousarray(np.asarray(a, dtype=np.float32)), device=device)


def _i32(a, device):
  return torch.as_tensor(np.ascontiguousarray(np.asarray(a).astype(np.int32)), device=device)


def nxn_geom_pairs(mjm, unfiltered=False):
  """Filtered NXN candidate pairs and pair ids (io.py:269-358); `unfiltered` returns every upper-triangle
  pair with its ids instead (the reference's m.nxn_geom_pair / m.nxn_pairid, -2 = never a contact)."""
  filterparent = not (mjm.opt.disableflags & DisableBit.FILTERPARENT)
  g1, g2 = np.triu_indices(mjm.ngeom, k=1)
  bodyid1, bodyid2 = mjm.geom_bodyid[g1], mjm.geom_bodyid[g2]
  weldid1, weldid2 = mjm.body_weldid[bodyid1], mjm.body_weldid[bodyid2]
  weld_parentid1 = mjm.body_weldid[mjm.body_parentid[weldid1]]
  weld_parentid2 = mjm.body_weldid[mjm.body_parentid[weldid2]]
  self_collision = weldid1 == weldid2
  parent_child = filterparent & (weldid1 != 0) & (weldid2 != 0) & ((weldid1 == weld_parentid2) | (weldid2 == weld_parentid1))
  mask = np.array((mjm.geom_contype[g1] & mjm.geom_conaffinity[g2]) | (mjm.geom_contype[g2] & mjm.geom_conaffinity[g1]), dtype=bool)
  exclude = np.isin((bodyid1 << 16) + bodyid2, getattr(mjm, "exclude_signature", np.zeros(0, dtype=np.int32)))
  pairid_contact = -np.ones(len(g1), dtype=np.int32)
  pairid_contact[~(mask & ~self_collision & ~parent_child & ~exclude)] = -2
  # explicit <contact><pair> entries (io.py:296-302): always candidates, parameters from the pair
  n = mjm.ngeom
  for i in range(getattr(mjm, "npair", 0)):
    a, b = sorted((int(mjm.pair_geom1[i]), int(mjm.pair_geom2[i])))
    pairid_contact[(a * (2 * n - a - 3)) // 2 + b - 1] = i
  pairid_collision = -np.ones(len(g1), dtype=np.int32)
  if unfiltered:
    return np.stack([g1, g2], axis=1).astype(np.int32), np.stack([pairid_contact, pairid_collision], axis=1).astype(np.int32)
  include = pairid_contact > -2
  pairs = np.stack([g1, g2], axis=1)[include].astype(np.int32)
  pairid = np.stack([pairid_contact, pairid_collision], axis=1)[include].astype(np.int32)
  return pairs, pairid


# real model fields: header name -> (attribute on Model, MjModel source attr)
def _model_attr(name):
  if name.startswith("opt_"):
    return ("opt", name[4:])
  if name.startswith("stat_"):
    return ("stat", name[5:])
  return (None, name)


_SUPPORTED_GEOMS = {types.GeomType.PLANE, types.GeomType.HFIELD, types.GeomType.SPHERE, types.GeomType.CAPSULE, types.GeomType.ELLIPSOID, types.GeomType.CYLINDER,
                    types.GeomType.BOX, types.GeomType.MESH}
# every CONVEX entry of the reference table (collision_driver.py:43-77): GJK / EPA (heightfield pairs: per
# grid prism, collision_convex.py:158-697)
_CONVEX_TABLE = {(1, 2), (1, 3), (1, 4), (1, 5), (1, 6), (1, 7), (2, 4), (2, 7), (3, 4), (3, 5), (3, 7), (4, 4), (4, 5), (4, 6), (4, 7), (5, 5), (5, 6), (5, 7), (6, 6), (6, 7), (7, 7)}
# PRIMITIVE entries (type-sorted), collision_primitive.py:1280-1300: in the forward kernel's narrowphase ...
_PRIMITIVE_PAIRS = {(0, 2), (0, 3), (0, 6), (2, 2), (2, 3), (3, 3), (2, 6), (3, 6)}
# ... and in the dense path's pre-pass (ccd_kernel, one pair per lane): plane-ellipsoid, plane-cylinder,
# sphere-cylinder and plane-mesh (plane_convex) -- the multi-point or rare ones kept out of the hot kernel
_PREPASS_PRIMITIVES = {(0, 4), (0, 5), (2, 5), (0, 7)}
_SUPPORTED_PAIRS = _PRIMITIVE_PAIRS | _PREPASS_PRIMITIVES | _CONVEX_TABLE
# pairs with a pre-pass record slot on the dense path (nxn_ccdid)
_CCD_PAIRS = _PREPASS_PRIMITIVES | _CONVEX_TABLE
# the sparse path computes every primitive in its collision kernel and runs the convex pairs in its own
# CCD pre-pass (mjw_sparse.hip)
_SPARSE_PAIRS = _PREPASS_PRIMITIVES
_SPARSE_CCD_PAIRS = _CONVEX_TABLE


def put_model(mjm, device=None) -> types.Model:
  """Creates a model on device (reference io.py:77-647)."""
  dev = _device(device)
  # feature checks (io.py:89-144): the MI355X path supports the primitive-geom dense subset
  for g in np.unique(mjm.geom_type):
    if int(g) not in _SUPPORTED_GEOMS:
      raise NotImplementedError(f"geom type {types.GeomType(int(g)).name} not supported.")
  if mjm.opt.integrator not in (types.IntegratorType.EULER, types.IntegratorType.RK4, types.IntegratorType.IMPLICITFAST):
    raise NotImplementedError(f"{types.IntegratorType(mjm.opt.integrator).name} is unsupported.")
  if mjm.opt.cone not in (types.ConeType.PYRAMIDAL, types.ConeType.ELLIPTIC):
    raise NotImplementedError(f"cone {int(mjm.opt.cone)} is unsupported.")
  if mjm.opt.solver not in (types.SolverType.CG, types.SolverType.NEWTON):
    raise NotImplementedError(f"{types.SolverType(mjm.opt.solver).name} is unsupported.")
  if getattr(mjm.opt, "noslip_iterations", 0) > 0:
    raise NotImplementedError("noslip solver not implemented.")
  # io.py:114-121: flags outside the reference's DisableBit / EnableBit sets (types.py:166-221)
  unsupported = int(mjm.opt.disableflags) & int(DisableBit.MIDPHASE | DisableBit.AUTORESET)
  if unsupported:
    raise NotImplementedError(f"{DisableBit(unsupported).name} is unsupported.")
  unsupported = int(mjm.opt.enableflags) & int(EnableBit.OVERRIDE | EnableBit.FWDINV)
  if unsupported:
    raise NotImplementedError(f"{EnableBit(unsupported).name} is unsupported.")
  sparse = is_sparse(mjm) or getattr(mjm, "nflex", 0) > 0
  if sparse:
    # the workgroup-per-world sparse / flex pipeline (csrc/mjw_sparse.hip) covers this subset
    if getattr(mjm, "nsensor", 0):
      # the sensor kernel (csrc/mjw_sensor.hip) stages a world's body / dof state in 64 KB of LDS
      if 37 * mjm.nbody + 14 * mjm.nv > 16384:
        raise NotImplementedError("sparse / flex models: sensors need 37 nbody + 14 nv <= 16384 in this build (the flex bodies exceed it).")
  for st in np.unique(getattr(mjm, "sensor_type", np.zeros(0, dtype=np.int32))):
    if int(st) not in types.SUPPORTED_SENSORS:
      raise NotImplementedError(f"sensor type {int(st)} is not supported by this build yet.")
  if not sparse and getattr(mjm, "neq", 0) and np.any(~np.isin(mjm.eq_type, (types.EqType.CONNECT, types.EqType.WELD, types.EqType.JOINT, types.EqType.TENDON))):
    raise NotImplementedError("only connect, weld, joint and tendon equality constraints are supported by this build yet.")
  pairs_chk, _ = nxn_geom_pairs(mjm)
  for g1, g2 in pairs_chk:
    t = tuple(sorted((int(mjm.geom_type[g1]), int(mjm.geom_type[g2]))))
    if t not in (_SUPPORTED_PAIRS | _SPARSE_PAIRS | _SPARSE_CCD_PAIRS if sparse else _SUPPORTED_PAIRS):
      names = tuple(types.GeomType(x).name for x in t)
      raise NotImplementedError(f"collision between {names[0]} and {names[1]} is not supported by this build yet.")
  if mjm.opt.disableflags & DisableBit.NATIVECCD and any(
      tuple(sorted((int(mjm.geom_type[a]), int(mjm.geom_type[b])))) == (6, 6) for a, b in pairs_chk):
    raise NotImplementedError("box-box with NATIVECCD disabled (primitive box_box) is not supported by this build yet.")
  # io.py:372-409: margins on the multi-contact pairs (box-box always, box-mesh / mesh-mesh under MULTICCD).
  # One deviation: the reference also rejects box-box *geom* margins under NATIVECCD, which rejects its own
  # apollo benchmark (the hand plates, margin 5e-4, BASELINE.json configs[3]); here those pairs run, and
  # ccd() takes them as it does every pair with a margin -- one EPA contact, no multi-contact
  # (collision_gjk.py:2336-2338).  Explicit <pair> margins keep the reference's check.
  multiccd = bool(mjm.opt.enableflags & EnableBit.MULTICCD)
  nativeccd_off = bool(mjm.opt.disableflags & DisableBit.NATIVECCD)
  kinds_chk = [tuple(sorted((int(mjm.geom_type[a]), int(mjm.geom_type[b])))) for a, b in pairs_chk]
  if (6, 6) in kinds_chk or (multiccd and ((6, 7) in kinds_chk or (7, 7) in kinds_chk)) or int(getattr(mjm, "npair", 0)):
    def _check_margin(name, t1, t2, margin, explicit=False):
      if multiccd:
        raise NotImplementedError(f"{name} has non-zero margin ({margin}) with MULTICCD enabled. Set margin to 0 or disable MULTICCD.")
      if explicit and t1 in boxmesh and t2 in boxmesh and not nativeccd_off:
        raise NotImplementedError(f"{name} has non-zero margin ({margin}) with NATIVECCD enabled. Set margin to 0 or disable NATIVECCD.")

    boxmesh = (types.GeomType.BOX, types.GeomType.MESH)
    pair_set = {(int(a), int(b)) for a, b in zip(getattr(mjm, "pair_geom1", []), getattr(mjm, "pair_geom2", []))}
    for g1, g2 in pairs_chk:
      if (int(g1), int(g2)) in pair_set or (int(g2), int(g1)) in pair_set:
        continue
      t1, t2 = int(mjm.geom_type[g1]), int(mjm.geom_type[g2])
      m1, m2 = float(mjm.geom_margin[g1]), float(mjm.geom_margin[g2])
      if (m1 or m2) and t1 in boxmesh and t2 in boxmesh:
        _check_margin(f"geom pair ({g1}, {g2})", t1, t2, (m1, m2))
    for pid in range(int(getattr(mjm, "npair", 0))):
      t1, t2 = int(mjm.geom_type[mjm.pair_geom1[pid]]), int(mjm.geom_type[mjm.pair_geom2[pid]])
      if mjm.pair_margin[pid] and t1 in boxmesh and t2 in boxmesh:
        _check_margin(f"pair {pid}", t1, t2, float(mjm.pair_margin[pid]), explicit=True)
  muscle = _muscle_mask(mjm)
  if np.any(muscle):
    lr = np.asarray(mjm.actuator_lengthrange, np.float64).reshape(-1, 2)[muscle]
    if np.any(lr[:, 0] >= lr[:, 1]):
      raise NotImplementedError("muscle actuators need an actuator_lengthrange (lengthrange attribute, or a limited joint / tendon transmission).")
  if (mjm.opt.viscosity > 0 or mjm.opt.density > 0) and mjm.opt.integrator in (types.IntegratorType.IMPLICITFAST, types.IntegratorType.IMPLICIT):
    raise NotImplementedError("Implicit integrators and fluid model not implemented.")  # io.py:126-130

  nv = mjm.nv
  opt = types.Option()
  o = mjm.opt
  opt.timestep = _f32([o.timestep], dev)
  opt.tolerance = _f32([max(o.tolerance, 1e-6)], dev)  # io.py:185
  opt.ls_tolerance = _f32([o.ls_tolerance], dev)
  opt.ccd_tolerance = _f32([getattr(o, "ccd_tolerance", 1e-6)], dev)
  opt.ccd_iterations = int(getattr(o, "ccd_iterations", 35))
  opt.density = _f32([o.density], dev)
  opt.viscosity = _f32([o.viscosity], dev)
  opt.gravity = _f32(np.asarray(o.gravity).reshape(1, 3), dev)
  opt.wind = _f32(np.asarray(o.wind).reshape(1, 3), dev)
  opt.magnetic = _f32(np.asarray(o.magnetic).reshape(1, 3), dev)
  opt.impratio_invsqrt = _f32([1.0 / np.sqrt(max(o.impratio, types.MJ_MINVAL))], dev)  # io.py:178-179
  opt.integrator, opt.cone, opt.solver, opt.jacobian = int(o.integrator), int(o.cone), int(o.solver), int(o.jacobian)
  opt.iterations, opt.ls_iterations = int(o.iterations), int(o.ls_iterations)
  opt.disableflags, opt.enableflags = int(o.disableflags), int(o.enableflags)
  # io.py:188-190: the parallel linesearch switch (a <numeric name="ls_parallel"> of 1) and its smallest step
  opt.ls_parallel = bool(getattr(o, "ls_parallel", False))
  opt.ls_parallel_min_step = _f32([1.0e-6], dev)
  opt.contact_sensor_maxmatch = int(getattr(o, "contact_sensor_maxmatch", 64))  # io.py:195-199
  stat = types.Statistic(meaninertia=_f32([mjm.stat.meaninertia], dev))

  m = types.Model()
  m.opt = opt
  m.stat = stat
  m.callback = types.Callback()
  m.device = dev
  for n in ("nq", "nv", "nu", "na", "nbody", "njnt", "ngeom", "nsite", "ncam", "nlight", "nmocap", "nM", "nC"):
    setattr(m, n, int(getattr(mjm, n)))
  m.ntendon = int(getattr(mjm, "ntendon", 0))
  m.npair = int(getattr(mjm, "npair", 0))
  m.nwrap, m.nJten = int(getattr(mjm, "nwrap", 0)), int(getattr(mjm, "nJten", 0))
  m.ten_maxnnz = int(np.max(mjm.ten_J_rownnz)) if m.ntendon else 0  # the reference's max_ten_J_rownnz (io.py:232)
  # spatial tendons (smooth.py:3172-3465): their count selects the per-world length / Jacobian path; the
  # pulley divisor of each wrap (io.py:491-497)
  wrap_type = np.asarray(getattr(mjm, "wrap_type", np.zeros(0)), dtype=np.int32)
  m.nten_spatial = int(sum(wrap_type[mjm.tendon_adr[t]] != types.WrapType.JOINT for t in range(m.ntendon)))
  from .tendon_geom import pulley_scale

  wrap_pulley_scale = pulley_scale(mjm) if m.nwrap else np.zeros(0)
  m.nmuscle = int(np.sum(_muscle_mask(mjm)))  # > 0 selects the forward kernel compiled with the muscle paths
  # gravity compensation and fluid forces (passive.py:246-533; io.py:230, :2218-2219); either selects the
  # forward kernel's extended instantiation, as tendons and muscles do
  body_gravcomp = np.asarray(getattr(mjm, "body_gravcomp", np.zeros(mjm.nbody)), dtype=np.float64).reshape(-1, mjm.nbody)
  m.ngravcomp = int((body_gravcomp > 0.0).any(axis=0).sum())
  m.has_fluid = bool(np.any(np.asarray(o.wind) != 0) or o.density > 0 or o.viscosity > 0)
  geom_fluid = np.asarray(getattr(mjm, "geom_fluid", np.zeros((mjm.ngeom, 12))), dtype=np.float64).reshape(mjm.ngeom, 12)
  body_fluid_ellipsoid = np.zeros(mjm.nbody, dtype=np.int32)  # io.py:262-263
  body_fluid_ellipsoid[np.asarray(mjm.geom_bodyid)[geom_fluid[:, 0] > 0]] = 1
  # the sparse path's dense Newton Hessian (nv x nv per world), zero-sized otherwise
  m.sp_nH = int(mjm.nv) if (is_sparse(mjm) or getattr(mjm, "nflex", 0) > 0) and mjm.opt.solver == types.SolverType.NEWTON else 0
  m.neq = int(getattr(mjm, "neq", 0))
  m.nsensor = int(getattr(mjm, "nsensor", 0))
  m.nsensordata = int(getattr(mjm, "nsensordata", 0))
  stypes = np.asarray(getattr(mjm, "sensor_type", np.zeros(0, dtype=np.int32)))
  m.sensor_rne_postconstraint = int(np.isin(stypes, list(types.RNE_POSTCONSTRAINT_SENSORS)).any())  # io.py:542-551
  m.nsensor_acc = int((np.asarray(getattr(mjm, "sensor_needstage", np.zeros(0))) == types.Stage.ACC).sum())
  m.is_sparse = bool(sparse)
  njmax_pad_unused, m.nv_pad = _padded_sizes(nv, 0, False)
  m.nmaxcondim = int(np.concatenate(([0], mjm.geom_condim, getattr(mjm, "pair_dim", []))).max())
  m.nmaxpyramid = int(max(1, 2 * (m.nmaxcondim - 1)))
  m.block_dim = None

  # derived tree arrays (io.py:234-258): levels; DFS subtree ranges (bodies are in DFS pre-order)
  depth = np.zeros(mjm.nbody, dtype=int)
  for i in range(1, mjm.nbody):
    depth[i] = depth[mjm.body_parentid[i]] + 1
  order = np.argsort(depth, kind="stable")
  m.nlevel = int(depth.max()) + 1 if mjm.nbody else 0
  level_adr = np.searchsorted(depth[order], np.arange(m.nlevel + 1))
  subtree_end = np.arange(mjm.nbody) + 1
  for i in range(mjm.nbody - 1, 0, -1):
    p = mjm.body_parentid[i]
    subtree_end[p] = max(subtree_end[p], subtree_end[i])
  m.body_tree = tuple(torch.as_tensor(order[level_adr[i] : level_adr[i + 1]].astype(np.int32), device=dev) for i in range(m.nlevel))
  # host-side sanity: DFS pre-order is required for subtree ranges
  for i in range(1, mjm.nbody):
    assert mjm.body_parentid[i] < i, "bodies must be in DFS pre-order"

  jnt_limited_sh = np.nonzero(mjm.jnt_limited & np.isin(mjm.jnt_type, (JointType.SLIDE, JointType.HINGE)))[0]
  jnt_limited_ball = np.nonzero(mjm.jnt_limited & (mjm.jnt_type == JointType.BALL))[0]
  pairs, pairid = nxn_geom_pairs(mjm)
  typed = pairs.copy()
  swap = mjm.geom_type[typed[:, 0]] > mjm.geom_type[typed[:, 1]]
  typed[swap] = typed[swap][:, ::-1]
  m.nxn_geom_pair_filtered = _i32(pairs, dev)
  m.nxn_pairid_filtered = _i32(pairid, dev)
  pairs_all, pairid_all = nxn_geom_pairs(mjm, unfiltered=True)  # the reference's unfiltered fields (API parity)
  m.nxn_geom_pair, m.nxn_pairid = _i32(pairs_all, dev), _i32(pairid_all, dev)
  m.nxn_geom_pair_typed = _i32(typed, dev)
  m.nxn = len(pairs)
  kinds = [tuple(sorted((int(mjm.geom_type[a]), int(mjm.geom_type[b])))) for a, b in pairs]
  ccd_set = _SPARSE_CCD_PAIRS if sparse else _CCD_PAIRS
  m.nxn_ccd = int(sum(k in ccd_set for k in kinds))
  # pairs that need the forward kernel's box / pre-pass narrowphase paths (the BOX instantiation)
  m.nxn_box = int(sum((6 in k) or (k in ccd_set) for k in kinds))
  ccdid = np.cumsum([k in ccd_set for k in kinds]) - 1
  m.nxn_ccdid = _i32(np.where([k in ccd_set for k in kinds], ccdid, -1) if kinds else np.zeros(0), dev)
  m.nmesh, m.nmeshvert = int(getattr(mjm, "nmesh", 0)), int(getattr(mjm, "nmeshvert", 0))
  m.nhfield, m.nhfielddata = int(getattr(mjm, "nhfield", 0)), int(getattr(mjm, "nhfielddata", 0))
  m.nmeshpoly, m.nmeshpolyvert = int(getattr(mjm, "nmeshpoly", 0)), int(getattr(mjm, "nmeshpolyvert", 0))
  m.nmeshnormal = int(getattr(mjm, "nmeshnormal", 0))
  m.nmeshpolymap = int(getattr(mjm, "nmeshpolymap", 0))
  # multi-contact workspace (collision_convex.py:1120-1140): 4-gon faces / 3 normals per vertex for box-box;
  # with MULTICCD and box-mesh / mesh-mesh pairs the meshes' largest polygon and vertex degree
  mesh_multi = bool(mjm.opt.enableflags & EnableBit.MULTICCD) and any(
    tuple(sorted((int(mjm.geom_type[a]), int(mjm.geom_type[b])))) in ((6, 7), (7, 7)) for a, b in nxn_geom_pairs(mjm)[0])
  m.nmaxpolygon = max(4, int(np.max(mjm.mesh_polyvertnum))) if mesh_multi and m.nmeshpoly else 4
  m.nmaxmeshdeg = max(3, int(np.max(mjm.mesh_polymapnum))) if mesh_multi and m.nmeshpoly else 3
  m.nlimited = len(jnt_limited_sh)
  m.nlimited_ball = len(jnt_limited_ball)
  m.neq_cw = int(np.isin(mjm.eq_type, (types.EqType.CONNECT, types.EqType.WELD)).sum()) if mjm.neq else 0
  m.act_maxnnz = max([_mom_nnz(mjm, a) for a in range(mjm.nu)] + [0])
  m.nbodytrn = int(np.sum(np.asarray(mjm.actuator_trntype) == types.TrnType.BODY)) if mjm.nu else 0  # the reference's nacttrnbody
  m.nsitetrn = int(np.isin(np.asarray(mjm.actuator_trntype), (types.TrnType.SITE, types.TrnType.SLIDERCRANK)).sum()) if mjm.nu else 0

  m.nJmom = int(sum(_mom_nnz(mjm, a) for a in range(mjm.nu)))
  sc_adr, sc_num, sc_pair = _sensor_collision_pairs(mjm, pairid_all)
  # io.py:556-567: one taxel per vertex of each tactile sensor's mesh (global vertex index, sensor id)
  taxel_vertadr, taxel_sensorid = [], []
  for s_ in range(int(getattr(mjm, "nsensor", 0))):
    if int(mjm.sensor_type[s_]) == types.SensorType.TACTILE:
      mid = int(mjm.sensor_objid[s_])
      taxel_vertadr += [int(mjm.mesh_vertadr[mid]) + j for j in range(int(mjm.mesh_vertnum[mid]))]
      taxel_sensorid += [s_] * int(mjm.mesh_vertnum[mid])
  m.nsensortaxel = len(taxel_vertadr)
  m.nsensorcontact = int(sum(int(mjm.sensor_type[s_]) == types.SensorType.CONTACT for s_ in range(int(getattr(mjm, "nsensor", 0)))))
  m.nsensorcollision = len(sc_pair) // 4
  sc_kinds = [tuple(sorted((int(mjm.geom_type[a]), int(mjm.geom_type[b])))) for a, b in sc_pair.reshape(-1, 4)[:, :2]]
  m.nsensorccd = int(sum(k in _SENSOR_CONVEX or k in _SENSOR_HFIELD for k in sc_kinds))  # records the sensor kernel runs in lockstep
  # collision_convex.py:1127: EPA iteration cap over the convex pairs of the collision and sensor pair lists
  geom_pairs = {tuple(sorted(map(int, p_))) for p_ in pairs} | {tuple(sorted(map(int, r_[:2]))) for r_ in sc_pair.reshape(-1, 4)}
  gkinds = [tuple(sorted((int(mjm.geom_type[a]), int(mjm.geom_type[b])))) for a, b in geom_pairs]
  nconvex = sum(k in _CONVEX_TABLE for k in gkinds)
  nboxbox = sum(k == (6, 6) for k in gkinds)
  m.ccd_epa_iterations = 16 if nconvex and nboxbox == nconvex else int(getattr(mjm.opt, "ccd_iterations", 35))
  if m.nsensorccd and 37 * mjm.nbody + 14 * mjm.nv + _ccd_words(m.ccd_epa_iterations, m.nmaxpolygon, m.nmaxmeshdeg) + 368 * (m.nhfield > 0) + 32 * m.nsensorcollision > 16384:
    raise NotImplementedError("collision sensors on convex pairs: the sensor kernel's 64 KB of LDS is exceeded by this model.")

  # sparse path: kinematic trees as dof ranges (a tree starts at every dof without a parent dof),
  # J row width = the longest union of two dof chains (+ the 6 dofs of a flex edge)
  dof_parent = np.asarray(mjm.dof_parentid)
  starts = np.nonzero(dof_parent < 0)[0] if nv else np.zeros(0, dtype=int)
  tree_dofadr = np.concatenate([starts, [nv]]).astype(np.int32)
  chain = np.zeros(nv, dtype=int)
  for i in range(nv):
    chain[i] = 1 + (chain[dof_parent[i]] if dof_parent[i] >= 0 else 0)
  maxchain = int(chain.max()) if nv else 0
  m.ntree = len(starts)
  nflex = int(getattr(mjm, "nflex", 0))
  # tendon rows (friction, limit: one tendon's Jacobian row; equality: the union of two) fit a J row too
  ten_w = int(max(mjm.ten_J_rownnz)) if getattr(mjm, "ntendon", 0) else 0
  for e in range(int(getattr(mjm, "neq", 0))):
    if mjm.eq_type[e] == types.EqType.TENDON and mjm.eq_obj2id[e] >= 0:
      ten_w = max(ten_w, int(mjm.ten_J_rownnz[mjm.eq_obj1id[e]] + mjm.ten_J_rownnz[mjm.eq_obj2id[e]]))
  m.njrow = max(2 * maxchain, 6 if nflex else 0, 2, ten_w) if sparse else m.nv_pad
  # flex collision candidates (collision_flex.py:381-529 tests every sphere / capsule / box / cylinder
  # geom whose contype / conaffinity matches) and planes (:261-378)
  cg_adr, cg = [0], []
  for f in range(nflex):
    for g in range(mjm.ngeom):
      if int(mjm.geom_type[g]) in (2, 3, 5, 6) and ((mjm.geom_contype[g] & mjm.flex_conaffinity[f]) or (mjm.flex_contype[f] & mjm.geom_conaffinity[g])):
        cg.append(g)
    cg_adr.append(len(cg))
  planes = np.nonzero(mjm.geom_type == 0)[0] if nflex else np.zeros(0, dtype=int)
  # per-vertex contribution lists of the flex passive forces: element vertex slots (4 per element, the
  # first dim + 1 used), then bending slots (4 per edge)
  nfv = int(getattr(mjm, "nflexvert", 0))
  inc = [[] for _ in range(nfv)]
  for f in range(nflex):
    vb = mjm.flex_vertadr[f]
    nve = int(mjm.flex_dim[f]) + 1
    for el in range(mjm.flex_elemnum[f]):
      eg = mjm.flex_elemadr[f] + el
      for k in range(nve):
        inc[vb + mjm.flex_elem[mjm.flex_elemdataadr[f] + nve * el + k]].append(4 * eg + k)
  nelem = int(getattr(mjm, "nflexelem", 0))
  for f in range(nflex):
    vb = mjm.flex_vertadr[f]
    for e in range(mjm.flex_edgeadr[f], mjm.flex_edgeadr[f] + mjm.flex_edgenum[f]):
      if mjm.flex_edgeflap[e, 1] < 0:
        continue
      vs = (mjm.flex_edge[e, 0], mjm.flex_edge[e, 1], mjm.flex_edgeflap[e, 0], mjm.flex_edgeflap[e, 1])
      for k, v in enumerate(vs):
        inc[vb + v].append(4 * nelem + 4 * e + k)
  inc_adr = np.concatenate([[0], np.cumsum([len(x) for x in inc])]).astype(np.int32)
  inc_flat = np.array([c for x in inc for c in x], dtype=np.int32)
  m.nflex, m.nflexvert, m.nflexedge = nflex, nfv, int(getattr(mjm, "nflexedge", 0))
  m.nflexelem, m.nflexelemdata = nelem, int(getattr(mjm, "nflexelemdata", 0))
  m.nflexelemedge = int(getattr(mjm, "nflexelemedge", 3 * nelem))
  m.nflexshelldata = int(getattr(mjm, "nflexshelldata", 0))
  m.nflexinc, m.nflexcg, m.nplane = len(inc_flat), len(cg), len(planes)
  derived_int = dict(
    tree_dofadr=tree_dofadr,
    body_fluid_ellipsoid=body_fluid_ellipsoid,
    flex_cgeomadr=np.array(cg_adr, dtype=np.int32),
    flex_cgeom=np.array(cg, dtype=np.int32),
    plane_geom=planes.astype(np.int32),
    flexvert_incadr=inc_adr,
    flexvert_inc=inc_flat,
    body_subtree_end=subtree_end,
    body_level=depth,
    level_body=order,
    level_adr=level_adr,
    jnt_limited_slide_hinge_adr=jnt_limited_sh,
    jnt_limited_ball_adr=jnt_limited_ball,
    taxel_vertadr=np.array(taxel_vertadr, dtype=np.int32),
    taxel_sensorid=np.array(taxel_sensorid, dtype=np.int32),
    sensor_collision_adr=sc_adr,
    sensor_collision_num=sc_num,
    sensor_collision_pair=sc_pair,
  )
  for k_, v_ in derived_int.items():
    if k_ in ("tree_dofadr", "flex_cgeomadr", "flex_cgeom", "plane_geom", "flexvert_incadr", "flexvert_inc", "body_fluid_ellipsoid",
              "taxel_vertadr", "taxel_sensorid",
              "sensor_collision_adr", "sensor_collision_num", "sensor_collision_pair"):
      setattr(m, k_, _i32(v_, dev))
  m.body_subtree_end = _i32(subtree_end, dev)
  m.body_level = _i32(depth, dev)
  m.level_body = _i32(order, dev)
  m.level_adr = _i32(level_adr, dev)
  m.jnt_limited_slide_hinge_adr = _i32(jnt_limited_sh, dev)
  m.jnt_limited_ball_adr = _i32(jnt_limited_ball, dev)

  # real arrays (batched with leading dim 1)
  for name, cnt in _lib.MODEL_REAL_ARRAYS:
    grp, attr = _model_attr(name)
    if grp is not None:
      continue
    val = np.asarray(wrap_pulley_scale if name == "wrap_pulley_scale" else getattr(mjm, attr), dtype=np.float64)
    setattr(m, attr, _f32(val.reshape((1,) + val.shape), dev))
  for name, cnt in _lib.MODEL_INT_ARRAYS:
    if name in derived_int or name in ("nxn_geom_pair", "nxn_pairid", "nxn_ccdid"):
      continue
    setattr(m, name, _i32(np.asarray(getattr(mjm, name)), dev))
  # extra reference fields kept for API parity
  for name in ("dof_Madr", "M_rownnz", "M_rowadr", "M_colind", "mapM2M", "body_geomnum", "body_geomadr", "geom_contype", "geom_conaffinity", "exclude_signature",
               "eq_active0", "body_mocapid"):
    if hasattr(mjm, name):
      setattr(m, name, _i32(np.asarray(getattr(mjm, name)), dev))
  m._mjm_sizes = dict(nq=mjm.nq, nv=nv)
  return m


# collision sensors (GEOMDIST / GEOMNORMAL / GEOMFROMTO) and the pairs they can evaluate: the type-sorted
# pairs of collision_driver.py:43-77's PRIMITIVE entries, in the sensor kernel's primitive narrowphase ...
_COLLISION_SENSORS = (types.SensorType.GEOMDIST, types.SensorType.GEOMNORMAL, types.SensorType.GEOMFROMTO)
# ... and the convex entries (heightfields aside), GJK / EPA with an unbounded cutoff in the sensor kernel
_SENSOR_CONVEX = {k for k in _CONVEX_TABLE if k[0] != 1}
_SENSOR_HFIELD = {k for k in _CONVEX_TABLE if k[0] == 1}  # ... and heightfields (the prism routine)
_SENSOR_PAIRS = _PRIMITIVE_PAIRS | {(0, 4), (0, 5), (2, 5)} | _SENSOR_CONVEX | _SENSOR_HFIELD


def _ccd_words(it, npoly=4, ndeg=3):
  """Words of mjw_ccd.h's lockstep GJK / EPA workspace (ccd_layout, no heightfield scratch)."""
  cv, cf = 10 + 2 * it, 6 + 5 * it
  npoly, ndeg = max(npoly, 4), max(ndeg, 3)
  nclip = max(2 * npoly, 16)
  return cv * 4 + cf * 5 + 24 + 36 + 8 + 4 + 2 * 20 + 32 + 12 + 12 + 6 * ndeg + 2 * ndeg + 3 * ndeg + 3 * npoly * 3 + npoly + 6 * nclip


def _sensor_collision_pairs(mjm, pairid_all):
  """Per collision sensor, the geom pairs it collides (io.py:304-346: every geom of obj (a geom, or a body's
  geoms) against every geom of ref, in that loop order) as (g1, g2, pairid, flip) records with (g1, g2)
  in the narrowphase's type-then-index order, pairid the explicit <pair> that sets the margin (-1: the geoms'
  margins), and flip = the record's order is (ref, obj) (sensor.py:656-661).  Returns (adr, num, flat
  records); adr = -1 for the other sensors."""
  ns = int(getattr(mjm, "nsensor", 0))
  adr, num, recs = np.full(ns, -1, np.int32), np.zeros(ns, np.int32), []
  n = mjm.ngeom
  for s_ in range(ns):
    if int(mjm.sensor_type[s_]) not in _COLLISION_SENSORS:
      continue
    geoms = []
    for ot, oid in ((mjm.sensor_objtype[s_], mjm.sensor_objid[s_]), (mjm.sensor_reftype[s_], mjm.sensor_refid[s_])):
      if int(ot) == types.ObjType.BODY:
        geoms.append(range(mjm.body_geomadr[oid], mjm.body_geomadr[oid] + mjm.body_geomnum[oid]))
      else:
        geoms.append([int(oid)])
    adr[s_] = len(recs)
    for a in geoms[0]:
      for b in geoms[1]:
        if a == b:
          raise NotImplementedError(f"collision sensor {s_}: a geom against itself")
        ta, tb = int(mjm.geom_type[a]), int(mjm.geom_type[b])
        if tuple(sorted((ta, tb))) not in _SENSOR_PAIRS:
          names = tuple(types.GeomType(x).name for x in sorted((ta, tb)))
          raise NotImplementedError(f"collision sensor {s_}: {names[0]}-{names[1]} is not in the collision table")
        flip = ta > tb or (ta == tb and a > b)
        g1, g2 = (b, a) if flip else (a, b)
        lo, hi = min(a, b), max(a, b)
        pid = int(pairid_all[(lo * (2 * n - lo - 3)) // 2 + hi - 1, 0])
        recs.append((g1, g2, max(pid, -1), int(flip)))
        num[s_] += 1
  return adr, num, np.array(recs, dtype=np.int32).reshape(-1)


def _mom_nnz(mjm, a) -> int:
  """Non-zeros of actuator a's moment row, as smooth.py:2042-2442 counts them: the joint's dofs, the tendon's
  Jacobian row, the union of the two sites' weld-body dof chains (SLIDERCRANK; SITE with a reference site stops
  at their common ancestor dof), one site's chain (SITE), or every dof (BODY)."""
  trn, (i1, i2) = int(mjm.actuator_trntype[a]), mjm.actuator_trnid[a]
  if trn == types.TrnType.TENDON:
    return int(mjm.ten_J_rownnz[i1])
  if trn == types.TrnType.BODY:
    return int(mjm.nv)
  if trn in (types.TrnType.SITE, types.TrnType.SLIDERCRANK):
    last = lambda s_: (lambda b: mjm.body_dofadr[b] + mjm.body_dofnum[b] - 1 if b > 0 else -1)(mjm.body_weldid[mjm.site_bodyid[s_]])
    d1 = last(i1)
    d2 = last(i2) if i2 >= 0 else -1
    n = 0
    while d1 >= 0 or d2 >= 0:
      da = max(d1, d2)
      if trn == types.TrnType.SITE and i2 >= 0 and d1 == da and d2 == da:
        break
      n += 1
      if d1 == da:
        d1 = mjm.dof_parentid[d1]
      if d2 == da:
        d2 = mjm.dof_parentid[d2]
    return n
  return {JointType.FREE: 6, JointType.BALL: 3}.get(int(mjm.jnt_type[i1]), 1)


# derived topology the C views carry beyond the reference Model fields
DERIVED_INT_ARRAYS = {
  "body_subtree_end": "body_subtree_end", "body_level": "body_level", "level_body": "level_body", "level_adr": "level_adr",
  "jnt_limited_slide_hinge_adr": "jnt_limited_slide_hinge_adr", "jnt_limited_ball_adr": "jnt_limited_ball_adr",
  "nxn_geom_pair": "nxn_geom_pair_typed", "nxn_pairid": "nxn_pairid_filtered", "nxn_ccdid": "nxn_ccdid",
  "tree_dofadr": "tree_dofadr", "flex_cgeomadr": "flex_cgeomadr", "flex_cgeom": "flex_cgeom", "plane_geom": "plane_geom",
  "flexvert_incadr": "flexvert_incadr", "flexvert_inc": "flexvert_inc",
  "sensor_collision_adr": "sensor_collision_adr", "sensor_collision_num": "sensor_collision_num", "sensor_collision_pair": "sensor_collision_pair",
  "taxel_vertadr": "taxel_vertadr", "taxel_sensorid": "taxel_sensorid",
}
DERIVED_SCALARS = ("act_maxnnz", "nbodytrn", "nsitetrn", "nten_spatial", "nxn", "nxn_ccd", "nxn_box", "ccd_epa_iterations", "nlevel", "nlimited", "nlimited_ball", "neq_cw", "nJmom", "ntree", "njrow", "ten_maxnnz", "nmuscle", "sp_nH",
                   "nv_pad", "nmaxcondim", "nmaxpyramid", "sensor_rne_postconstraint", "nsensor_acc", "nflexinc", "nflexcg", "nplane",
                   "nsensorcollision", "nsensorccd", "nsensortaxel", "nsensorcontact")


def derive_model_fields(mjm) -> dict:
  """Host helper for a reference-side binding: the derived index arrays and sizes of mjw_model_t that the
  reference Model does not hold (DFS subtree ends, level lists, filtered / type-sorted NXN pairs, convex-pair
  ids, sparse-path tree and flex incidence lists), computed from MjModel fields exactly as put_model does.
  Returns {name: int32 numpy array or int}; the caller uploads the arrays once."""
  m = put_model(mjm, device="cpu")
  out = {name: getattr(m, attr).numpy().astype(np.int32).copy() for name, attr in DERIVED_INT_ARRAYS.items()}
  out.update({name: int(getattr(m, name)) for name in DERIVED_SCALARS})
  return out


def _nb(t: torch.Tensor):
  return int(t.shape[0])


def cmodel(m: types.Model) -> _lib.CModel:
  """Builds (and caches) the C model view holding the device pointers of `m`."""
  tensors = []
  for name, _ in _lib.MODEL_REAL_ARRAYS:
    grp, attr = _model_attr(name)
    t = getattr(getattr(m, grp), attr) if grp else getattr(m, attr)
    if not isinstance(t, torch.Tensor):  # an Option scalar set as a Python number (e.g. ls_parallel_min_step)
      t = torch.tensor([float(t)], dtype=torch.float32, device=m.device)
      setattr(getattr(m, grp) if grp else m, attr, t)
    tensors.append(t)
  for name, _ in _lib.MODEL_INT_ARRAYS:
    attr = {"nxn_geom_pair": "nxn_geom_pair_typed", "nxn_pairid": "nxn_pairid_filtered"}.get(name, name)
    tensors.append(getattr(m, attr))
  cache = getattr(m, "_cmodel_cache", None)
  scal = tuple(int(getattr(m.opt, n[4:]) if n.startswith("opt_") else getattr(m, n)) for n in _lib.MODEL_INT_SCALARS)
  if cache is not None and cache[1] == scal and len(cache[2]) == len(tensors) and all(a is b for a, b in zip(cache[2], tensors)):
    return cache[0]
  c = _lib.CModel()
  for n in _lib.MODEL_INT_SCALARS:
    if n.startswith("opt_"):
      v = int(getattr(m.opt, n[4:]))
    else:
      v = int(getattr(m, n))
    setattr(c, n, v)
  sizes = {n: getattr(c, n) for n in _lib.MODEL_INT_SCALARS}
  i = 0
  for name, cnt in _lib.MODEL_REAL_ARRAYS:
    t = tensors[i]
    i += 1
    if t.dtype != torch.float32 or not t.is_contiguous():
      raise TypeError(f"model field {name} must be a contiguous float32 tensor")
    count = int(eval(cnt, {}, sizes))
    nb = _nb(t) if t.dim() > 0 else 1
    if t.numel() != nb * count:
      raise ValueError(f"model field {name}: expected {count} values per batch entry, got shape {tuple(t.shape)}")
    setattr(c, name, t.data_ptr())
    setattr(c, name + "_nb", nb)
    setattr(c, name + "_cnt", count)
  for name, cnt in _lib.MODEL_INT_ARRAYS:
    t = tensors[i]
    i += 1
    count = int(eval(cnt, {}, sizes))
    if t.numel() != count:
      raise ValueError(f"model field {name}: expected {count} values, got {t.numel()}")
    setattr(c, name, t.data_ptr())
  m._cmodel_cache = (c, scal, tensors)
  return c


# Data field trailing shapes (types.py:1702-1896)
def _data_shapes(m, nworld, njmax, njmax_pad, naconmax):
  nb, nv, nq, nu, na, nj, ng = m.nbody, m.nv, m.nq, m.nu, m.na, m.njnt, m.ngeom
  sp = int(bool(m.is_sparse))
  np_ = m.nv_pad
  real = dict(
    time=(), qpos=(nq,), qvel=(nv,), act=(na,), ctrl=(nu,), qacc_warmstart=(nv,), qfrc_applied=(nv,),
    xfrc_applied=(nb, 6), mocap_pos=(m.nmocap, 3), mocap_quat=(m.nmocap, 4), qacc=(nv,), act_dot=(na,), energy=(2,),
    xpos=(nb, 3), xquat=(nb, 4), xmat=(nb, 3, 3), xipos=(nb, 3), ximat=(nb, 3, 3), xanchor=(nj, 3), xaxis=(nj, 3),
    geom_xpos=(ng, 3), geom_xmat=(ng, 3, 3), site_xpos=(m.nsite, 3), site_xmat=(m.nsite, 3, 3),
    cam_xpos=(m.ncam, 3), cam_xmat=(m.ncam, 3, 3), light_xpos=(m.nlight, 3), light_xdir=(m.nlight, 3),
    subtree_com=(nb, 3), subtree_linvel=(nb, 3), subtree_angmom=(nb, 3), cdof=(nv, 6), cinert=(nb, 10), crb=(nb, 10),
    qM=(m.nM,) if sp else (np_, np_), qLD=(m.nM,) if sp else (nv, nv),
    actuator_length=(nu,), actuator_moment=(m.nJmom,), actuator_velocity=(nu,), actuator_force=(nu,),
    cvel=(nb, 6), cdof_dot=(nv, 6), qfrc_bias=(nv,), qfrc_spring=(nv,), qfrc_damper=(nv,), qfrc_gravcomp=(nv,), qfrc_fluid=(nv,),
    qfrc_passive=(nv,), qfrc_actuator=(nv,), qfrc_smooth=(nv,), qacc_smooth=(nv,), qfrc_constraint=(nv,),
    cacc=(nb, 6), cfrc_int=(nb, 6), cfrc_ext=(nb, 6), sensordata=(m.nsensordata,), ccd_out=(m.nxn_ccd * 32,),
    efc_J=(m.njrow, njmax_pad) if sp else (njmax_pad, m.njrow), efc_pos=(njmax,), efc_margin=(njmax,), efc_D=(njmax_pad,), efc_vel=(njmax,),
    efc_aref=(njmax,), efc_frictionloss=(njmax,), efc_force=(njmax,), efc_Ma=(nv,),
    # RK4 workspace (forward.py:462-472 temporaries; kept resident so a step allocates nothing)
    qpos_t0=(nq,), qvel_t0=(nv,), act_t0=(na,), qvel_rk=(nv,), qacc_rk=(nv,), act_dot_rk=(na,),
    # flex (smooth.py:228-355) and the sparse path's workspace (size 0 on the dense path)
    flexvert_xpos=(m.nflexvert, 3), flexedge_length=(m.nflexedge,), flexedge_velocity=(m.nflexedge,),
    flexedge_J=(m.nflexedge, 6), flex_frc=(m.nflexelem * 12 + m.nflexedge * 12,),
    sp_body=(nb * 6 * sp,), sp_vec=(nv * 10 * sp,), sp_row=(njmax * 3 * sp,), sp_LD=(m.nM * sp,),
    sp_H=(m.sp_nH * m.sp_nH,),
    efc_JT_val=(njmax_pad * m.njrow * sp,),
    # fixed tendons (smooth.py:3085-3121): lengths, velocities, sparse Jacobian (ten_J_rowadr / _colind)
    ten_length=(m.ntendon,), ten_velocity=(m.ntendon,), ten_J=(m.nJten,),
  )
  ints = dict(
    ne=(), nf=(), nl=(), nefc=(), solver_niter=(), moment_rownnz=(nu,), moment_rowadr=(nu,), moment_colind=(m.nJmom,),
    efc_type=(njmax,), efc_id=(njmax,), efc_state=(njmax_pad,), eq_active=(m.neq,),
    efc_J_colind=(m.njrow * sp, njmax_pad), efc_J_rownnz=(njmax * sp,), efc_JT_rowind=(njmax_pad * m.njrow * sp,),
    efc_JT_adr=((nv + 1) * sp,), sp_cnt=((nv + 1) * sp,), ncon_world=(2,), sp_idx16=(njmax_pad * m.njrow * sp,),
    # the dense path's longest-first world order (mjw_step.hip) and each world's iteration bucket
    world_order=(), world_key=(),
  )
  creal = dict(
    contact_dist=(), contact_pos=(3,), contact_frame=(3, 3), contact_includemargin=(), contact_friction=(5,),
    contact_solref=(2,), contact_solreffriction=(2,), contact_solimp=(5,),
  )
  cint = dict(contact_dim=(), contact_geom=(2,), contact_efc_address=(m.nmaxpyramid,), contact_worldid=(), contact_type=(), contact_geomcollisionid=(),
              contact_flex=(2,), contact_vert=(2,))
  return real, ints, creal, cint


def _valid_sizes():
  return (2 + (np.arange(19) % 2)) * (2 ** (np.arange(19) // 2 + 3))


def _default_nconmax(mjm, mjd=None) -> int:
  """io.py:664-674."""
  nconmax = max(mjm.nv * 0.35 * (getattr(mjm, "nhfield", 0) > 0) * 10 + 45, getattr(mjd, "ncon", 0) if mjd is not None else 0)
  vs = _valid_sizes()
  return int(vs[np.searchsorted(vs, nconmax)])


def _default_njmax(mjm, mjd=None) -> int:
  """io.py:677-687."""
  njmax = max(mjm.nv * 2.26 * (getattr(mjm, "nhfield", 0) > 0) * 18 + 53, getattr(mjd, "nefc", 0) if mjd is not None else 0)
  vs = _valid_sizes()
  return int(vs[np.searchsorted(vs, njmax)])


def _resolve_batch_size(na, n, nworld, default):
  """io.py:850-855."""
  if na is not None:
    return na
  if n is not None:
    return n * nworld
  return default


def _alloc_data(m, nworld, nconmax, njmax, naconmax, device, nccdmax=None, njmax_nnz=None, naccdmax=None):
  """Sizes and checks of make_data (io.py:885-932), then the device arrays.

  nccdmax / naccdmax bound the convex (GJK/EPA) contacts in the reference's separate CCD pool; here the
  convex pre-pass writes into a fixed per-pair slot (Data.ccd_out) and its contacts join the one pool, so
  they are validated and recorded only.  njmax_nnz (sparse J non-zeros) is recorded: the sparse path keeps
  efc_J slot-major with a fixed row width m.njrow, so njmax * njrow values are allocated."""
  if nworld < 1:
    raise ValueError("nworld must be >= 1")
  if nconmax is None:
    nconmax = _default_nconmax(m)
  if njmax is None:
    njmax = _default_njmax(m)
  if nconmax < 0:
    raise ValueError("nconmax must be >= 0")
  if njmax < 0:
    raise ValueError("njmax must be >= 0")
  naconmax = _resolve_batch_size(naconmax, nconmax, nworld, 0)
  if naconmax < 0:
    raise ValueError("naconmax must be >= 0")
  naccdmax = _resolve_batch_size(naccdmax, nccdmax, nworld, naconmax)
  if naccdmax < 0:
    raise ValueError("naccdmax must be >= 0")
  elif naccdmax > naconmax:
    raise ValueError(f"naccdmax ({naccdmax}) must be <= naconmax ({naconmax})")
  if nccdmax is None:
    nccdmax = nconmax
  elif nccdmax < 0:
    raise ValueError("nccdmax must be >= 0")
  elif nccdmax > nconmax:
    raise ValueError(f"nccdmax ({nccdmax}) must be <= nconmax ({nconmax})")
  if njmax_nnz is None:
    njmax_nnz = njmax * m.nv
  njmax_pad, _ = _padded_sizes(m.nv, njmax, False)
  if m.is_sparse and (njmax_pad > 65536 or m.nv > 65535):
    # the sparse CG keeps its row / dof indices in 16 bits (sp_idx16, csrc/mjw_sparse.hip)
    raise NotImplementedError(f"sparse / flex models: njmax ({njmax}) must be <= 65536 and nv ({m.nv}) <= 65535 in this build.")
  real, ints, creal, cint = _data_shapes(m, nworld, njmax, njmax_pad, naconmax)
  d = types.Data()
  d.nworld, d.njmax, d.njmax_pad, d.naconmax, d.nconmax = nworld, njmax, njmax_pad, naconmax, nconmax
  d.njmax_nnz, d.nccdmax, d.naccdmax = int(njmax_nnz), int(nccdmax), int(naccdmax)
  d.world_offset = 0
  d.device = device
  d.efc = types.Constraint()
  d.contact = types.Contact()
  for name, shp in real.items():
    t = torch.zeros((nworld,) + shp, dtype=torch.float32, device=device)
    _set_data_field(d, name, t)
  for name, shp in ints.items():
    t = torch.zeros((nworld,) + shp, dtype=torch.int32, device=device)
    _set_data_field(d, name, t)
  for name, shp in creal.items():
    _set_data_field(d, name, torch.zeros((naconmax,) + shp, dtype=torch.float32, device=device))
  for name, shp in cint.items():
    _set_data_field(d, name, torch.zeros((naconmax,) + shp, dtype=torch.int32, device=device))
  d.contact.efc_address.fill_(-1)
  # nacon and ncollision adjacent (one 8-B aligned allocation): the dense step kernel adds a world's
  # broadphase pairs and its contact slots with one 64-bit atomic (mjw_step.hip collision_and_constraints)
  counters = torch.zeros(2, dtype=torch.int32, device=device)
  d.nacon = counters[0:1]
  d.ncollision = counters[1:2]
  # MJW_SCHED=0: no longest-first world order for the dense kernel (A/B runs)
  d.sched = None if os.environ.get("MJW_SCHED") == "0" else torch.zeros(_lib.SCHED_WORDS, dtype=torch.int32, device=device)
  d.efc.J_rowadr = torch.zeros((nworld, 0), dtype=torch.int32, device=device)
  d.mocap_quat[..., 0] = 1.0
  d.xquat[..., 0] = 1.0
  return d


def _set_data_field(d, name, t):
  if name.startswith("efc_") and name != "efc_Ma":
    setattr(d.efc, name[4:], t)
  elif name == "efc_Ma":
    d.efc.Ma = t
  elif name.startswith("contact_"):
    setattr(d.contact, name[8:], t)
  else:
    setattr(d, name, t)


def _get_data_field(d, name):
  if name.startswith("efc_"):
    return getattr(d.efc, name[4:])
  if name.startswith("contact_"):
    return getattr(d.contact, name[8:])
  return getattr(d, name)


def cdata(d: types.Data) -> _lib.CData:
  """Builds (and caches) the C data view holding the device pointers of `d`."""
  names = [n for n, _ in _lib.DATA_REAL_ARRAYS + _lib.DATA_INT_ARRAYS + _lib.CONTACT_REAL_ARRAYS + _lib.CONTACT_INT_ARRAYS]
  tensors = [_get_data_field(d, n) for n in names] + [d.nacon, d.ncollision, d.sched]
  cache = getattr(d, "_cdata_cache", None)
  key = (d.nworld, d.njmax, d.njmax_pad, d.naconmax, d.world_offset)
  if cache is not None and cache[1] == key and all(a is b for a, b in zip(cache[2], tensors)):
    return cache[0]
  c = _lib.CData()
  c.nworld, c.njmax, c.njmax_pad, c.naconmax, c.world_offset = key
  for n, t in zip(names, tensors):
    if not t.is_contiguous():
      raise TypeError(f"data field {n} must be contiguous")
    setattr(c, n, t.data_ptr())
  c.nacon = d.nacon.data_ptr()
  c.ncollision = d.ncollision.data_ptr()
  # world-order workspace; None -> the dense kernels run the worlds in identity order
  c.sched = d.sched.data_ptr() if d.sched is not None else None
  d._cdata_cache = (c, key, tensors)
  return c


def make_data(mjm, nworld: int = 1, nconmax: Optional[int] = None, nccdmax: Optional[int] = None, njmax: Optional[int] = None,
              njmax_nnz: Optional[int] = None, naconmax: Optional[int] = None, naccdmax: Optional[int] = None, device=None,
              m: Optional[types.Model] = None) -> types.Data:
  """Creates a data object on device (io.py:859-868) initialised to qpos0 / zero state."""
  dev = _device(device)
  if m is None:
    m = put_model(mjm, device=dev)
  d = _alloc_data(m, nworld, nconmax, njmax, naconmax, dev, nccdmax=nccdmax, njmax_nnz=njmax_nnz, naccdmax=naccdmax)
  d.qpos[:] = torch.as_tensor(np.asarray(mjm.qpos0, dtype=np.float32), device=dev)
  if m.neq:  # int32 on the device (the reference's bool), initialised from eq_active0
    d.eq_active[:] = torch.as_tensor(np.asarray(mjm.eq_active0, dtype=np.int32), device=dev)
  if mjm.nmocap:
    for b in np.nonzero(mjm.body_mocapid >= 0)[0]:
      k = mjm.body_mocapid[b]
      d.mocap_pos[:, k] = torch.as_tensor(np.asarray(mjm.body_pos[b], dtype=np.float32), device=dev)
      d.mocap_quat[:, k] = torch.as_tensor(np.asarray(mjm.body_quat[b], dtype=np.float32), device=dev)
  return d


def put_data(mjm, mjd, nworld: int = 1, nconmax: Optional[int] = None, nccdmax: Optional[int] = None, njmax: Optional[int] = None, njmax_nnz: Optional[int] = None, naconmax: Optional[int] = None, naccdmax: Optional[int] = None, device=None, m: Optional[types.Model] = None) -> types.Data:
  """Moves one host state to the device, tiled over nworld worlds (io.py:1016-1240)."""
  dev = _device(device)
  if m is None:
    m = put_model(mjm, device=dev)
  if nconmax is None:
    nconmax = _default_nconmax(mjm, mjd)
  if njmax is None:
    njmax = _default_njmax(mjm, mjd)
  if nconmax < 0:
    raise ValueError("nconmax must be >= 0")
  if njmax < 0:
    raise ValueError("njmax must be >= 0")
  ncon = int(getattr(mjd, "ncon", 0))
  if naconmax is None and ncon > nconmax:
    raise ValueError(f"nconmax overflow (nconmax must be >= {ncon})")
  if int(getattr(mjd, "nefc", 0)) > njmax:
    raise ValueError(f"njmax overflow (njmax must be >= {mjd.nefc})")
  d = _alloc_data(m, nworld, nconmax, njmax, naconmax, dev, nccdmax=nccdmax, njmax_nnz=njmax_nnz, naccdmax=naccdmax)

  def tile(name, val, shape):
    if val is None:
      return
    arr = np.asarray(val, dtype=np.float64).reshape(shape)
    getattr(d, name)[:] = torch.as_tensor(arr.astype(np.float32), device=dev)

  tile("time", np.full(nworld, float(np.asarray(mjd.time).reshape(-1)[0] if np.ndim(mjd.time) else mjd.time)), (nworld,))
  tile("qpos", mjd.qpos, (mjm.nq,))
  tile("qvel", mjd.qvel, (mjm.nv,))
  tile("act", mjd.act, (mjm.na,))
  tile("ctrl", mjd.ctrl, (mjm.nu,))
  tile("qacc_warmstart", mjd.qacc_warmstart, (mjm.nv,))
  tile("qfrc_applied", mjd.qfrc_applied, (mjm.nv,))
  tile("xfrc_applied", mjd.xfrc_applied, (mjm.nbody, 6))
  if mjm.nmocap:
    tile("mocap_pos", mjd.mocap_pos, (mjm.nmocap, 3))
    tile("mocap_quat", mjd.mocap_quat, (mjm.nmocap, 4))
  if hasattr(mjd, "qacc"):
    tile("qacc", mjd.qacc, (mjm.nv,))
  if m.neq:
    eqa = getattr(mjd, "eq_active", mjm.eq_active0)
    d.eq_active[:] = torch.as_tensor(np.asarray(eqa, dtype=np.int32).reshape(m.neq), device=dev)
  d.solver_niter.fill_(int(np.asarray(getattr(mjd, "solver_niter", [0])).reshape(-1)[0]))
  return d


def get_data_into(result, mjm, d: types.Data, world_id: int = 0):
  """Copies one world of `d` into a host MjData-like object (io.py:1243-1455)."""
  if world_id < 0 or world_id >= d.nworld:
    raise ValueError(f"world_id {world_id} out of range")
  for name in ("qpos", "qvel", "act", "ctrl", "qacc_warmstart", "qfrc_applied", "qacc", "act_dot", "xpos", "xquat", "xipos", "xanchor",
               "xaxis", "geom_xpos", "site_xpos", "cam_xpos", "light_xpos", "light_xdir", "subtree_com", "cdof", "cinert", "crb",
               "actuator_length", "actuator_velocity", "actuator_force", "cvel", "cdof_dot", "qfrc_bias", "qfrc_spring", "qfrc_damper",
               "qfrc_gravcomp", "qfrc_fluid", "qfrc_passive", "qfrc_actuator", "qfrc_smooth", "qacc_smooth", "qfrc_constraint", "cacc", "cfrc_int",
               "cfrc_ext", "xfrc_applied", "mocap_pos", "mocap_quat", "energy", "sensordata"):
    if hasattr(result, name) or isinstance(result, object):
      val = getattr(d, name)[world_id].detach().cpu().numpy().astype(np.float64)
      try:
        cur = getattr(result, name)
        cur[...] = val.reshape(np.shape(cur))
      except AttributeError:
        setattr(result, name, val)
  for name in ("xmat", "ximat", "geom_xmat", "site_xmat", "cam_xmat"):
    val = getattr(d, name)[world_id].detach().cpu().numpy().astype(np.float64).reshape(-1, 9)
    try:
      cur = getattr(result, name)
      cur[...] = val.reshape(np.shape(cur))
    except AttributeError:
      setattr(result, name, val)
  result.time = float(d.time[world_id])
  nv = mjm.nv
  nefc = int(d.nefc[world_id])
  nrows = min(nefc, d.njmax)
  result.nefc = nefc
  if d.efc.J_colind.numel():  # sparse path: ancestor-row qM / qLD, slot-major J (densified here)
    qm = d.qM[world_id].detach().cpu().numpy().astype(np.float64)
    M = np.zeros((nv, nv))
    for i in range(nv):
      for k in range(mjm.M_rownnz[i]):
        j = mjm.M_colind[mjm.M_rowadr[i] + k]
        M[i, j] = M[j, i] = qm[mjm.M_rowadr[i] + k]
    result.qM_dense = M
    result.qLD_sparse = d.qLD[world_id].detach().cpu().numpy().astype(np.float64)
    vals = d.efc.J[world_id, :, :nrows].detach().cpu().numpy().astype(np.float64)
    cols = d.efc.J_colind[world_id, :, :nrows].cpu().numpy()
    nnz = d.efc.J_rownnz[world_id, :nrows].cpu().numpy()
    J = np.zeros((nrows, nv))
    for r in range(nrows):
      for k in range(nnz[r]):
        J[r, cols[k, r]] += vals[k, r]
    result.efc_J = J
  else:
    result.qM_dense = d.qM[world_id, :nv, :nv].detach().cpu().numpy().astype(np.float64)
    result.qLD_dense = d.qLD[world_id].detach().cpu().numpy().astype(np.float64)
    result.efc_J = d.efc.J[world_id, :nrows, :nv].detach().cpu().numpy().astype(np.float64)
  for f in ("pos", "margin", "D", "vel", "aref", "frictionloss", "force"):
    setattr(result, "efc_" + f, getattr(d.efc, f)[world_id, :nrows].detach().cpu().numpy().astype(np.float64))
  for f in ("type", "id", "state"):
    setattr(result, "efc_" + f, getattr(d.efc, f)[world_id, :nrows].detach().cpu().numpy())
  # contacts of this world, in pool order
  nacon = min(int(d.nacon[0]), d.naconmax)
  wid = d.contact.worldid[:nacon].detach().cpu().numpy()
  sel = np.nonzero(wid == world_id)[0]
  result.ncon = len(sel)
  result.contact = types.Contact(**{
    f: getattr(d.contact, f)[:nacon].detach().cpu().numpy()[sel]
    for f in ("dist", "pos", "frame", "includemargin", "friction", "solref", "solreffriction", "solimp", "dim", "geom", "efc_address")
  })
  result.solver_niter = np.array([int(d.solver_niter[world_id])])
  return result


def reset_data(m: types.Model, d: types.Data, reset: Optional[torch.Tensor] = None):
  """Clear data, set defaults; optionally by world (io.py:1458-1691).

  For every world where `reset` is True (all worlds when it is None): qpos <- qpos0 (batched, indexed by
  world), eq_active <- eq_active0, mocap_pos / mocap_quat <- body_pos / body_quat of the mocap bodies;
  qvel, act, ctrl, qacc_warmstart, qfrc_applied, xfrc_applied, qacc, act_dot, sensordata, energy, time, qM,
  solver_niter and the ne / nf / nl / nefc counters cleared; that world's contacts in the global pool
  cleared (efc_address -1, reset_contact :1575-1622).  The pool counter nacon is cleared only when world 0
  is reset (the reference does it from world 0's thread, :1558-1559), and after the contact clear
  (the clear reads nacon, :1577)."""
  dev = d.qpos.device
  mask = torch.ones(d.nworld, dtype=torch.bool, device=dev) if reset is None else reset.to(device=dev, dtype=torch.bool)
  if mask.shape != (d.nworld,):
    raise ValueError(f"reset mask must have shape ({d.nworld},), got {tuple(mask.shape)}")
  idx = torch.nonzero(mask).reshape(-1)
  if idx.numel() == 0:
    return
  gid = idx  # world ids of this Data (batched model fields are indexed worldid % nb)

  def _rows(t):
    return t[0] if t.shape[0] == 1 else t[gid % t.shape[0]]

  # contacts of the reset worlds (before nacon is touched)
  nacon = min(int(d.nacon[0]), d.naconmax)
  if nacon:
    wid = d.contact.worldid[:nacon].long()
    hit = torch.nonzero((wid < 0) | mask[wid.clamp(min=0)]).reshape(-1)
    if hit.numel():
      for f in ("dist", "pos", "frame", "includemargin", "friction", "solref", "solreffriction", "solimp", "dim", "geom", "flex", "vert",
                "worldid", "type", "geomcollisionid"):
        getattr(d.contact, f)[hit] = 0
      d.contact.efc_address[hit] = -1
  d.qpos[idx] = _rows(m.qpos0)
  for name in ("qvel", "act", "ctrl", "qacc_warmstart", "qfrc_applied", "xfrc_applied", "qacc", "act_dot", "sensordata", "energy", "qM"):
    t = getattr(d, name)
    if t.numel():
      t[idx] = 0
  for name in ("time", "solver_niter", "ne", "nf", "nl", "nefc"):
    getattr(d, name)[idx] = 0
  if d.eq_active.numel():
    d.eq_active[idx] = m.eq_active0.to(torch.int32)
  if d.mocap_pos.numel():
    bodies = torch.nonzero(m.body_mocapid >= 0).reshape(-1)
    mid = m.body_mocapid[bodies].long()
    bp, bq = _rows(m.body_pos), _rows(m.body_quat)  # (nbody, k) or (nreset, nbody, k)
    d.mocap_pos[idx.view(-1, 1), mid.view(1, -1)] = bp[..., bodies, :] if bp.dim() == 3 else bp[bodies].expand(idx.numel(), -1, -1)
    d.mocap_quat[idx.view(-1, 1), mid.view(1, -1)] = bq[..., bodies, :] if bq.dim() == 3 else bq[bodies].expand(idx.numel(), -1, -1)
  if bool(mask[0]):
    d.nacon.zero_()


def override_model(model, overrides: Sequence[str] | dict):
  """Applies 'opt.solver=cg' style overrides (io.py:2498-2588) to an MjModel or Model."""
  enums = {
    "solver": types.SolverType,
    "integrator": types.IntegratorType,
    "cone": types.ConeType,
    "jacobian": types.JacobianType,
  }
  items = overrides.items() if isinstance(overrides, dict) else [s.split("=", 1) for s in overrides]
  for key, val in items:
    key = key.strip()
    val = str(val).strip()
    obj = model
    parts = key.split(".")
    for p in parts[:-1]:
      obj = getattr(obj, p)
    leaf = parts[-1]
    if leaf in enums:
      v = int(enums[leaf][val.upper()])
    elif leaf in ("iterations", "ls_iterations", "disableflags", "enableflags", "ccd_iterations"):
      v = int(val)
    else:
      try:
        v = float(val)
      except ValueError:
        v = val
    cur = getattr(obj, leaf)
    if isinstance(cur, torch.Tensor):
      cur.fill_(float(v))
    else:
      setattr(obj, leaf, v)
  return model


def find_keys(model, keyname_prefix: str) -> list:
  """Ids of the keyframes whose name starts with `keyname_prefix`, in key order (io.py:2591-2600)."""
  return [k for k, name in enumerate(model.key_names) if name.startswith(keyname_prefix)]


def make_trajectory(model, keys: list) -> np.ndarray:
  """Control trajectory through the keys' ctrl values, linearly interpolated in time at opt.timestep
  (io.py:2603-2626): one row per step, the first key at time 0, keys in time order."""
  ctrls = []
  prev_ctrl = np.zeros(model.nu, dtype=np.float64)
  prev_time, time = 0.0, 0.0
  dt = float(model.opt.timestep)
  for key in keys:
    ctrl_key, ctrl_time = np.asarray(model.key_ctrl[key], dtype=np.float64), float(model.key_time[key])
    if not ctrls and ctrl_time != 0.0:
      raise ValueError("first keyframe must have time 0.0")
    if ctrls and ctrl_time <= prev_time:
      raise ValueError("keyframes must be in time order")
    while time < ctrl_time:
      frac = (time - prev_time) / (ctrl_time - prev_time)
      ctrls.append(prev_ctrl * (1 - frac) + ctrl_key * frac)
      time += dt
    ctrls.append(ctrl_key)
    time += dt
    prev_ctrl = ctrl_key
    prev_time = time
  return np.array(ctrls)
