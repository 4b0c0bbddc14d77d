"""ctypes binding of the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  It parses the X-macro field lists of oracle.h so the ctypes
structs match the C structs exactly, builds the oracle model from a host
`MjModel` (the NXN pair filter is restated independently of the product, from
mujoco_warp/_src/io.py:269-358), and runs the oracle over (nworld, ...) numpy
state arrays.
"""

from __future__ import annotations

import ctypes
import os
import re
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_BUILD = os.path.join(_HERE, "_build")


def build():
  subprocess.run(["make", "-s", "-C", _HERE], check=True)


def _macro_entries(text, macro):
  m = re.search(r"#define\s+" + macro + r"\(X\)(.*?)(?:\n\s*\n|\n/\*)", text, re.S)
  if not m:
    raise RuntimeError(f"macro {macro} not found in oracle.h")
  body = m.group(1).replace("\\\n", " ")
  return re.findall(r"X\(\s*([A-Za-z_0-9]+)\s*(?:,\s*([^)]*))?\)", body)


with open(os.path.join(_HERE, "oracle.h")) as f:
  _HDR = f.read()
MODEL_INT_SCALARS = [n for n, _ in _macro_entries(_HDR, "ORC_MODEL_INT_SCALARS")]
MODEL_REAL_SCALARS = [n for n, _ in _macro_entries(_HDR, "ORC_MODEL_REAL_SCALARS")]
MODEL_REAL_ARRAYS = _macro_entries(_HDR, "ORC_MODEL_REAL_ARRAYS")
MODEL_INT_ARRAYS = _macro_entries(_HDR, "ORC_MODEL_INT_ARRAYS")
DATA_REAL_ARRAYS = _macro_entries(_HDR, "ORC_DATA_REAL_ARRAYS")
DATA_INT_ARRAYS = _macro_entries(_HDR, "ORC_DATA_INT_ARRAYS")

_LIBS = {}


def _lib(real_bits):
  """real_bits 64 / 32, or "32f": fp32 with fused multiply-adds (liborc32f, the device's contraction)."""
  if real_bits not in _LIBS:
    path = os.path.join(_BUILD, f"liborc{real_bits}.so")
    if not os.path.exists(path):
      build()
    lib = ctypes.CDLL(path)
    _LIBS[real_bits] = lib
  return _LIBS[real_bits]


def _structs(real_bits):
  creal = ctypes.c_double if real_bits == 64 else ctypes.c_float
  mfields = [(n, ctypes.c_int) for n in MODEL_INT_SCALARS]
  mfields += [(n, creal) for n in MODEL_REAL_SCALARS]
  mfields += [(n, ctypes.POINTER(creal)) for n, _ in MODEL_REAL_ARRAYS]
  mfields += [(n, ctypes.POINTER(ctypes.c_int)) for n, _ in MODEL_INT_ARRAYS]
  dfields = [("njmax", ctypes.c_int), ("nconmax", ctypes.c_int)]
  dfields += [(n, ctypes.POINTER(creal)) for n, _ in DATA_REAL_ARRAYS]
  dfields += [(n, ctypes.POINTER(ctypes.c_int)) for n, _ in DATA_INT_ARRAYS]

  class OrcModel(ctypes.Structure):
    _fields_ = mfields

  class OrcData(ctypes.Structure):
    _fields_ = dfields

  return creal, OrcModel, OrcData


def nxn_pairs(mjm):
  """NXN candidate pair list (restatement of io.py:269-358, contact pairs only)."""
  ng = mjm.ngeom
  g1, g2 = np.triu_indices(ng, k=1)
  b1, b2 = mjm.geom_bodyid[g1], mjm.geom_bodyid[g2]
  w1, w2 = mjm.body_weldid[b1], mjm.body_weldid[b2]
  wp1 = mjm.body_weldid[mjm.body_parentid[w1]]
  wp2 = mjm.body_weldid[mjm.body_parentid[w2]]
  filterparent = not (mjm.opt.disableflags & (1 << 10))
  self_col = w1 == w2
  parent_child = filterparent & (w1 != 0) & (w2 != 0) & ((w1 == wp2) | (w2 == wp1))
  mask = ((mjm.geom_contype[g1] & mjm.geom_conaffinity[g2]) | (mjm.geom_contype[g2] & mjm.geom_conaffinity[g1])).astype(bool)
  excl = np.isin((b1 << 16) + b2, getattr(mjm, "exclude_signature", np.zeros(0, dtype=np.int32)))
  keep = mask & ~self_col & ~parent_child & ~excl
  pid = -np.ones(len(g1), dtype=np.int32)
  for i in range(getattr(mjm, "npair", 0)):  # explicit pairs (io.py:301-302): kept whatever the filters say
    a, b = sorted((int(mjm.pair_geom1[i]), int(mjm.pair_geom2[i])))
    k = int(np.nonzero((g1 == a) & (g2 == b))[0][0])
    keep[k] = True
    pid[k] = i
  pairs = np.stack([g1[keep], g2[keep]], axis=1).astype(np.int32)
  pairid = np.stack([pid[keep], -np.ones(keep.sum(), dtype=np.int32)], axis=1).astype(np.int32)
  return pairs, pairid


# convex (GJK/EPA) entries of MJ_COLLISION_TABLE (collision_driver.py:42-76), heightfield pairs included
CONVEX_PAIRS = {(1, 2), (1, 3), (1, 4), (1, 5), (1, 6), (1, 7),
                (2, 4), (2, 7), (3, 4), (3, 5), (3, 7), (4, 4), (4, 5), (4, 6), (4, 7), (5, 5), (5, 6), (5, 7), (6, 6), (6, 7), (7, 7)}


def _sensor_geom_pairs(mjm):
  """The geom pairs of the collision sensors (GEOMDIST / GEOMNORMAL / GEOMFROMTO: obj geoms x ref geoms)."""
  out = set()
  for s_ in range(int(getattr(mjm, "nsensor", 0))):
    if int(mjm.sensor_type[s_]) not in (39, 40, 41):
      continue
    sides = []
    for ot, oid in ((mjm.sensor_objtype[s_], mjm.sensor_objid[s_]), (mjm.sensor_reftype[s_], mjm.sensor_refid[s_])):
      sides.append(range(mjm.body_geomadr[oid], mjm.body_geomadr[oid] + mjm.body_geomnum[oid]) if int(ot) == 1 else [int(oid)])
    out |= {tuple(sorted((int(a), int(b)))) for a in sides[0] for b in sides[1]}
  return out


def ccd_epa_iterations(mjm, pairs):
  """EPA iteration cap: 16 when every convex pair -- of the collision and the collision-sensor pair lists --
  is box-box, else opt.ccd_iterations (collision_convex.py:1127)."""
  allpairs = {tuple(sorted((int(a), int(b)))) for a, b in pairs} | _sensor_geom_pairs(mjm)
  convex = [t for t in (tuple(sorted((int(mjm.geom_type[a]), int(mjm.geom_type[b])))) for a, b in allpairs) if t in CONVEX_PAIRS]
  nboxbox = sum(t == (6, 6) for t in convex)
  return 16 if convex and nboxbox == len(convex) else int(getattr(mjm.opt, "ccd_iterations", 35))


class OracleModel:
  """Oracle view of a host MjModel (one, unbatched model)."""

  def __init__(self, mjm, real_bits=64, overrides=None):
    self.real_bits = real_bits
    self.lib = _lib(real_bits)
    self.creal, self.StructM, self.StructD = _structs(real_bits)
    self.dtype = np.float64 if real_bits == 64 else np.float32
    self.mjm = mjm
    pairs, pairid = nxn_pairs(mjm)
    o = mjm.opt
    vals = dict(
      nq=mjm.nq, nv=mjm.nv, nu=mjm.nu, na=mjm.na, nbody=mjm.nbody, njnt=mjm.njnt, ngeom=mjm.ngeom, nsite=mjm.nsite,
      ncam=mjm.ncam, nlight=mjm.nlight, nmocap=mjm.nmocap, nxn=len(pairs), neq=mjm.neq,
      nsensor=getattr(mjm, "nsensor", 0), nsensordata=getattr(mjm, "nsensordata", 0),
      nmaxpyramid=max(1, 2 * (int(np.concatenate(([0], mjm.geom_condim, getattr(mjm, "pair_dim", []))).max()) - 1)),
      opt_integrator=o.integrator, opt_cone=o.cone, opt_solver=o.solver, opt_iterations=o.iterations,
      opt_ls_iterations=o.ls_iterations, opt_disableflags=o.disableflags, opt_enableflags=o.enableflags,
      opt_broadphase_filter=int(getattr(o, "broadphase_filter", 1 | 2 | 8)),
      opt_ccd_iterations=getattr(o, "ccd_iterations", 35), ccd_epa_iterations=ccd_epa_iterations(mjm, pairs),
      opt_ccd_tolerance=getattr(o, "ccd_tolerance", 1e-6),
      opt_timestep=o.timestep, opt_tolerance=max(o.tolerance, 1e-6), opt_ls_tolerance=o.ls_tolerance,
      opt_impratio_invsqrt=1.0 / np.sqrt(max(o.impratio, 1e-15)), stat_meaninertia=mjm.stat.meaninertia,
      is_sparse=int(getattr(mjm.opt, "jacobian", 2) == 1 or (getattr(mjm.opt, "jacobian", 2) == 2 and mjm.nv > 32)),
      nflex=getattr(mjm, "nflex", 0), nflexvert=getattr(mjm, "nflexvert", 0), nflexedge=getattr(mjm, "nflexedge", 0),
      nflexelem=getattr(mjm, "nflexelem", 0), nflexelemdata=getattr(mjm, "nflexelemdata", 0),
      nflexelemedge=getattr(mjm, "nflexelemedge", 3 * getattr(mjm, "nflexelem", 0)), nflexshelldata=getattr(mjm, "nflexshelldata", 0),
      nmeshnormal=getattr(mjm, "nmeshnormal", 0),
      nmesh=getattr(mjm, "nmesh", 0), nmeshvert=getattr(mjm, "nmeshvert", 0),
      nmeshpoly=getattr(mjm, "nmeshpoly", 0), nmeshpolyvert=getattr(mjm, "nmeshpolyvert", 0), nmeshpolymap=getattr(mjm, "nmeshpolymap", 0),
      ntendon=getattr(mjm, "ntendon", 0), nwrap=getattr(mjm, "nwrap", 0), nJten=getattr(mjm, "nJten", 0),
      npair=getattr(mjm, "npair", 0),
      nhfield=getattr(mjm, "nhfield", 0), nhfielddata=getattr(mjm, "nhfielddata", 0),
      # passive.py:829-851: gravity compensation / fluid switches (io.py:230, :2218-2219)
      ngravcomp=int((np.asarray(getattr(mjm, "body_gravcomp", np.zeros(mjm.nbody))) > 0).sum()),
      has_fluid=int(bool(np.any(np.asarray(o.wind) != 0) or o.density > 0 or o.viscosity > 0)),
      opt_density=o.density, opt_viscosity=o.viscosity,
      opt_ls_parallel=int(bool(getattr(o, "ls_parallel", False))), opt_contact_sensor_maxmatch=int(getattr(o, "contact_sensor_maxmatch", 64)), opt_ls_parallel_min_step=getattr(o, "ls_parallel_min_step", 1e-6),
    )
    if overrides:
      vals.update(overrides)
    self.sizes = {k: int(v) for k, v in vals.items() if k in MODEL_INT_SCALARS}
    geom_fluid = np.asarray(getattr(mjm, "geom_fluid", np.zeros((mjm.ngeom, 12))), dtype=np.float64).reshape(mjm.ngeom, 12)
    fluid_ellipsoid = np.zeros(mjm.nbody, dtype=np.int32)  # io.py:262-263
    fluid_ellipsoid[np.asarray(mjm.geom_bodyid)[geom_fluid[:, 0] > 0]] = 1
    arrays = dict(
      opt_gravity=o.gravity, opt_magnetic=o.magnetic, opt_wind=o.wind, nxn_geom_pair=pairs, nxn_pairid=pairid,
      body_gravcomp=getattr(mjm, "body_gravcomp", np.zeros(mjm.nbody)), geom_fluid=geom_fluid, body_fluid_ellipsoid=fluid_ellipsoid,
      cam_mat0=getattr(mjm, "cam_mat0", np.zeros((mjm.ncam, 9))),
      sensor_intprm=getattr(mjm, "sensor_intprm", np.zeros((getattr(mjm, "nsensor", 0), 3))),
    )
    self._keep = []
    s = self.StructM()
    for n in MODEL_INT_SCALARS:
      setattr(s, n, int(vals[n]))
    for n in MODEL_REAL_SCALARS:
      setattr(s, n, float(vals[n]))
    for n, cnt in MODEL_REAL_ARRAYS:
      a = arrays[n] if n in arrays else getattr(mjm, n)
      a = np.ascontiguousarray(np.asarray(a, dtype=self.dtype).reshape(-1))
      assert a.size == eval(cnt, {}, self.sizes), (n, a.size)
      self._keep.append(a)
      setattr(s, n, a.ctypes.data_as(ctypes.POINTER(self.creal)))
    for n, cnt in MODEL_INT_ARRAYS:
      a = arrays[n] if n in arrays else getattr(mjm, n)
      a = np.ascontiguousarray(np.asarray(a).astype(np.int32).reshape(-1))
      assert a.size == eval(cnt, {}, self.sizes), (n, a.size)
      self._keep.append(a)
      setattr(s, n, a.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
    self.struct = s
    self.nxn = len(pairs)


class OracleData:
  """(nworld, ...) numpy state/output arrays driven by the oracle."""

  def __init__(self, om: OracleModel, nworld: int, njmax: int, nconmax: int):
    self.om = om
    self.nworld, self.njmax, self.nconmax = nworld, njmax, nconmax
    sizes = dict(om.sizes, njmax=njmax, nconmax=nconmax)
    self.arrays = {}
    s = om.StructD()
    s.njmax, s.nconmax = njmax, nconmax
    for n, cnt in DATA_REAL_ARRAYS:
      a = np.zeros((nworld, max(eval(cnt, {}, sizes), 0)), dtype=om.dtype)
      self.arrays[n] = a
      setattr(s, n, a.ctypes.data_as(ctypes.POINTER(om.creal)))
    for n, cnt in DATA_INT_ARRAYS:
      a = np.zeros((nworld, max(eval(cnt, {}, sizes), 0)), dtype=np.int32)
      self.arrays[n] = a
      setattr(s, n, a.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
    self.struct = s
    m = om.mjm
    self.arrays["qpos"][:] = m.qpos0
    if m.nmocap:  # make_data (io.py:859-1013): mocap poses start at the mocap bodies' body_pos / body_quat
      self.arrays["mocap_quat"][:] = np.tile([1.0, 0, 0, 0], m.nmocap)
      for b in np.nonzero(np.asarray(m.body_mocapid) >= 0)[0]:
        k = int(m.body_mocapid[b])
        self.arrays["mocap_pos"][:, 3 * k:3 * k + 3] = m.body_pos[b]
        self.arrays["mocap_quat"][:, 4 * k:4 * k + 4] = m.body_quat[b]
    if m.neq:
      self.arrays["eq_active"][:] = np.asarray(m.eq_active0, dtype=np.int32)

  def __getattr__(self, name):
    arrays = self.__dict__.get("arrays")
    if arrays is not None and name in arrays:
      return arrays[name]
    raise AttributeError(name)

  def _call(self, fn, *extra):
    getattr(self.om.lib, fn)(ctypes.byref(self.om.struct), ctypes.byref(self.struct), ctypes.c_int(self.nworld), *extra)

  def step(self, nthread=1):
    self._call("orc_step", ctypes.c_int(nthread))

  def forward(self, nthread=1):
    self._call("orc_forward", ctypes.c_int(nthread))

  def fwd_position(self):
    self._call("orc_fwd_position")

  def fwd_position_polygons(self, cap=64):
    """fwd_position, returning the clipped polygons (> 4 vertices) polygon_quad searched: a list of
    (kept quad indices, (np, 3) vertices), in the order the narrowphase clipped them."""
    lib = self.om.lib
    real = ctypes.c_double if self.om.real_bits == 64 else ctypes.c_float
    stride = lib.orc_polylog_stride()
    buf = (real * (stride * cap))()
    lib.orc_polylog(buf, ctypes.c_int(cap))
    try:
      self.fwd_position()
      n = lib.orc_polylog_count()
    finally:
      lib.orc_polylog(None, ctypes.c_int(0))
    a = np.frombuffer(buf, dtype=np.float64 if self.om.real_bits == 64 else np.float32).reshape(cap, stride)[:n].astype(np.float64)
    return [(a[i, 1:5].astype(int), a[i, 5:5 + 3 * int(a[i, 0])].reshape(-1, 3)) for i in range(n)]

  def fwd_velocity(self):
    self._call("orc_fwd_velocity")

  def fwd_actuation(self):
    self._call("orc_fwd_actuation")

  def fwd_acceleration(self):
    self._call("orc_fwd_acceleration")

  def solve(self):
    self._call("orc_solve")

  def euler(self):
    self._call("orc_euler")

  def ctrl_noise(self, step, center=None, std=0.01, rate=0.1, world_offset=0):
    om = self.om
    c = np.zeros(0, dtype=om.dtype) if center is None else np.ascontiguousarray(center, dtype=om.dtype)
    om.lib.orc_ctrl_noise(
      ctypes.byref(om.struct),
      self.arrays["ctrl"].ctypes.data_as(ctypes.POINTER(om.creal)),
      c.ctypes.data_as(ctypes.POINTER(om.creal)),
      ctypes.c_int(c.size),
      ctypes.c_int(step),
      om.creal(std),
      om.creal(rate),
      ctypes.c_int(self.nworld),
      ctypes.c_int(world_offset),
    )


def kat_closest_segment_points(a0, a1, b0, b1, real_bits=64):
  lib = _lib(real_bits)
  creal = ctypes.c_double if real_bits == 64 else ctypes.c_float
  dt = np.float64 if real_bits == 64 else np.float32
  args = [np.ascontiguousarray(x, dtype=dt) for x in (a0, a1, b0, b1)]
  ba, bb = np.zeros(3, dt), np.zeros(3, dt)
  lib.orc_closest_segment_to_segment_points(*[x.ctypes.data_as(ctypes.POINTER(creal)) for x in args + [ba, bb]])
  return ba, bb


def kat_upper_tri_index(n, i, j):
  return _lib(64).orc_upper_tri_index(n, i, j)


def kat_upper_trid_index(n, i, j):
  return _lib(64).orc_upper_trid_index(n, i, j)


def kat_ccd(types, pos, mat, size, margin, tolerance, iterations, multiccd, mesh_vert=None, vertadr=(0, 0), vertnum=(0, 0),
            real_bits=64, mjm=None, meshid=None):
  """collision_gjk_test.py _geom_dist on the oracle: (ncon, dist, x1, x2); ncon -1 = not restated.  With the
  compiled model `mjm` and the geoms' mesh ids, mesh geoms carry their polygon data (mesh multi-contact)."""
  lib = _lib(real_bits)
  creal = ctypes.c_double if real_bits == 64 else ctypes.c_float
  dt = np.float64 if real_bits == 64 else np.float32
  P = lambda a: a.ctypes.data_as(ctypes.POINTER(creal))
  I = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_int))
  t = np.ascontiguousarray(types, dtype=np.int32)
  pos, mat, size = (np.ascontiguousarray(x, dtype=dt).reshape(-1) for x in (pos, mat, size))
  mv = np.ascontiguousarray(np.zeros(3) if mesh_vert is None else mesh_vert, dtype=dt).reshape(-1)
  va, vn = np.ascontiguousarray(vertadr, dtype=np.int32), np.ascontiguousarray(vertnum, dtype=np.int32)
  out = np.zeros(7, dt)
  if mjm is not None:
    om = OracleModel(mjm, real_bits=real_bits)
    mid = np.ascontiguousarray(meshid, dtype=np.int32)
    f = lib.orc_kat_ccd_model
    f.restype = ctypes.c_int
    n = f(I(t), P(pos), P(mat), P(size), P(mv), I(va), I(vn), creal(margin), creal(tolerance), ctypes.c_int(iterations),
          ctypes.c_int(int(multiccd)), ctypes.byref(om.struct), I(mid), P(out))
  else:
    f = lib.orc_kat_ccd
    f.restype = ctypes.c_int
    n = f(I(t), P(pos), P(mat), P(size), P(mv), I(va), I(vn), creal(margin), creal(tolerance), ctypes.c_int(iterations),
          ctypes.c_int(int(multiccd)), P(out))
  return n, float(out[0]), out[1:4].copy(), out[4:7].copy()


def kat_hfield_support(prism, direction, margin=0.0, real_bits=64):
  """collision_gjk_test.py:811-880 on the oracle: (support point, vertex index) of a heightfield prism."""
  lib = _lib(real_bits)
  creal = ctypes.c_double if real_bits == 64 else ctypes.c_float
  dt = np.float64 if real_bits == 64 else np.float32
  P = lambda a: a.ctypes.data_as(ctypes.POINTER(creal))
  pr = np.ascontiguousarray(prism, dtype=dt).reshape(-1)
  dr = np.ascontiguousarray(direction, dtype=dt).reshape(-1)
  out = np.zeros(3, dt)
  f = lib.orc_kat_hfield_support
  f.restype = ctypes.c_int
  vi = f(P(pr), P(dr), creal(margin), P(out))
  return out, int(vi)


def kat_wrap(fn, args, ind=0, radius=0.0, real_bits=64):
  """util_misc_test.py on the oracle: fn 'is_intersect' | 'length_circle' | 'wrap_circle' | 'wrap_inside' | 'wrap'."""
  lib = _lib(real_bits)
  creal = ctypes.c_double if real_bits == 64 else ctypes.c_float
  dt = np.float64 if real_bits == 64 else np.float32
  k = ["is_intersect", "length_circle", "wrap_circle", "wrap_inside", "wrap"].index(fn)
  a = np.ascontiguousarray(np.concatenate([np.ravel(x) for x in args]), dtype=dt)
  out = np.zeros(7, dt)
  f = lib.orc_kat_wrap
  f.restype = ctypes.c_int
  assert f(ctypes.c_int(k), a.ctypes.data_as(ctypes.POINTER(creal)), ctypes.c_int(int(ind)), creal(radius),
           out.ctypes.data_as(ctypes.POINTER(creal))) == 0
  if k < 2:
    return float(out[0])
  n = 2 if k < 4 else 3
  return float(out[0]), out[1:1 + n].copy(), out[1 + n:1 + 2 * n].copy()


def efc_row_params(disableflags, timestep, pos_aref, pos_imp, invweight, solref, solimp, vel):
  """(D, aref) of constraint rows from their inputs (constraint.py:52-121, fp64 oracle), vectorised over rows:
  pos_aref / pos_imp / invweight / vel of shape (n,), solref (n, 2), solimp (n, 5)."""
  lib = _lib(64)
  P = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))  # noqa: E731
  n = len(pos_aref)
  out = np.zeros((n, 2))
  sr = np.ascontiguousarray(solref, dtype=np.float64).reshape(n, 2)
  si = np.ascontiguousarray(solimp, dtype=np.float64).reshape(n, 5)
  o = np.zeros(2)
  for i in range(n):
    lib.orc_kat_efc_row(ctypes.c_int(int(disableflags)), ctypes.c_double(timestep), ctypes.c_double(pos_aref[i]),
                        ctypes.c_double(pos_imp[i]), ctypes.c_double(invweight[i]), P(sr[i]), P(si[i]), ctypes.c_double(vel[i]), P(o))
    out[i] = o
  return out[:, 0], out[:, 1]


def kat_geom_triangle(gt, gp, gr, gs, tri, tr, real_bits=64):
  """collision_primitive_core_test.py on the oracle: (n, out[2, 7] = dist, pos, normal)."""
  lib = _lib(real_bits)
  creal = ctypes.c_double if real_bits == 64 else ctypes.c_float
  dt = np.float64 if real_bits == 64 else np.float32
  P = lambda a: a.ctypes.data_as(ctypes.POINTER(creal))
  gp, gr, gs, tri = (np.ascontiguousarray(x, dtype=dt).reshape(-1) for x in (gp, gr, gs, tri))
  out = np.zeros(14, dt)
  f = lib.orc_kat_geom_triangle
  f.restype = ctypes.c_int
  n = f(ctypes.c_int(gt), P(gp), P(gr), P(gs), P(tri), creal(tr), P(out))
  return n, out.reshape(2, 7).copy()


def halton(index, base):
  f = _lib(64).orc_halton
  f.restype = ctypes.c_double
  return f(ctypes.c_int(index), ctypes.c_int(base))
