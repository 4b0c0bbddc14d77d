"""MJCF -> host model compiler (numpy, fp64).

mujoco_warp's `put_model` consumes a compiled `mujoco.MjModel`
(`mujoco_warp/_src/io.py:77-647`).  The MuJoCo C compiler is not available in
this image, so this module compiles the MJCF subset used by the benchmark
models into an `MjModel`-shaped host object with MuJoCo's field names and
conventions:

* defaults classes / childclass inheritance, degree->radian conversion;
* body / joint / dof / geom / site / camera / light / actuator / keyframe tables;
* inertia from geoms (mass = density * volume, capsule/sphere/box/... inertia,
  principal axes), `fromto` geom frames;
* derived tree arrays (rootid, weldid, dof_parentid, dof_Madr, M CSR layout);
* qpos0-dependent constants computed exactly like the reference's
  `set_const_0` (`io.py:2222-2407`): `stat.meaninertia`, `dof_invweight0`,
  `body_invweight0`, `cam/light *0`, `actuator_acc0`.

`put_model` also accepts a real `mujoco.MjModel` (duck typed) when the
`mujoco` package is importable.
"""

from __future__ import annotations

import copy
import math
import os
import xml.etree.ElementTree as ET
from typing import Optional

import numpy as np

from .types import (
  BiasType,
  CamLightType,
  ConeType,
  DataType,
  DisableBit,
  DynType,
  EnableBit,
  EqType,
  GainType,
  GeomType,
  IntegratorType,
  JacobianType,
  JointType,
  ObjType,
  SensorType,
  SolverType,
  Stage,
  TrnType,
  WrapType,
)

MJ_MINVAL = 1e-15

_DISABLE_NAMES = {
  "constraint": DisableBit.CONSTRAINT,
  "equality": DisableBit.EQUALITY,
  "frictionloss": DisableBit.FRICTIONLOSS,
  "limit": DisableBit.LIMIT,
  "contact": DisableBit.CONTACT,
  "spring": DisableBit.SPRING,
  "damper": DisableBit.DAMPER,
  "gravity": DisableBit.GRAVITY,
  "clampctrl": DisableBit.CLAMPCTRL,
  "warmstart": DisableBit.WARMSTART,
  "filterparent": DisableBit.FILTERPARENT,
  "actuation": DisableBit.ACTUATION,
  "refsafe": DisableBit.REFSAFE,
  "sensor": DisableBit.SENSOR,
  "midphase": DisableBit.MIDPHASE,
  "eulerdamp": DisableBit.EULERDAMP,
  "autoreset": DisableBit.AUTORESET,
  "nativeccd": DisableBit.NATIVECCD,
  "island": DisableBit.ISLAND,
}
_ENABLE_NAMES = {
  "override": EnableBit.OVERRIDE,
  "energy": EnableBit.ENERGY,
  "fwdinv": EnableBit.FWDINV,
  "invdiscrete": EnableBit.INVDISCRETE,
  "multiccd": EnableBit.MULTICCD,
}
_GEOM_TYPES = {
  "plane": GeomType.PLANE,
  "hfield": GeomType.HFIELD,
  "sphere": GeomType.SPHERE,
  "capsule": GeomType.CAPSULE,
  "ellipsoid": GeomType.ELLIPSOID,
  "cylinder": GeomType.CYLINDER,
  "box": GeomType.BOX,
  "mesh": GeomType.MESH,
  "sdf": GeomType.SDF,
}
_JOINT_TYPES = {"free": JointType.FREE, "ball": JointType.BALL, "slide": JointType.SLIDE, "hinge": JointType.HINGE}
_CAMLIGHT_MODES = {
  "fixed": CamLightType.FIXED,
  "track": CamLightType.TRACK,
  "trackcom": CamLightType.TRACKCOM,
  "targetbody": CamLightType.TARGETBODY,
  "targetbodycom": CamLightType.TARGETBODYCOM,
}
_INTEGRATORS = {
  "euler": IntegratorType.EULER,
  "rk4": IntegratorType.RK4,
  "implicit": IntegratorType.IMPLICIT,
  "implicitfast": IntegratorType.IMPLICITFAST,
}
_SOLVERS = {"pgs": SolverType.PGS, "cg": SolverType.CG, "newton": SolverType.NEWTON}
_CONES = {"pyramidal": ConeType.PYRAMIDAL, "elliptic": ConeType.ELLIPTIC}
_JACOBIANS = {"dense": JacobianType.DENSE, "sparse": JacobianType.SPARSE, "auto": JacobianType.AUTO}
_ACTUATOR_TAGS = ("motor", "position", "velocity", "general", "intvelocity", "damper", "muscle", "adhesion")

# MuJoCo default element attribute values (MJCF reference defaults).
_GEOM_DEFAULTS = dict(
  type="sphere",
  contype=1,
  conaffinity=1,
  condim=3,
  group=0,
  priority=0,
  size=[0.0, 0.0, 0.0],
  friction=[1.0, 0.005, 0.0001],
  solmix=1.0,
  solref=[0.02, 1.0],
  solimp=[0.9, 0.95, 0.001, 0.5, 2.0],
  margin=0.0,
  gap=0.0,
  density=1000.0,
)
_JOINT_DEFAULTS = dict(
  type="hinge",
  pos=[0.0, 0.0, 0.0],
  axis=[0.0, 0.0, 1.0],
  stiffness=0.0,
  damping=0.0,
  armature=0.0,
  frictionloss=0.0,
  springref=0.0,
  ref=0.0,
  margin=0.0,
  solreflimit=[0.02, 1.0],
  solimplimit=[0.9, 0.95, 0.001, 0.5, 2.0],
  solreffriction=[0.02, 1.0],
  solimpfriction=[0.9, 0.95, 0.001, 0.5, 2.0],
  limited="auto",
  range=[0.0, 0.0],
  actuatorfrclimited="auto",
  actuatorfrcrange=[0.0, 0.0],
  actuatorgravcomp="false",
)


def _floats(s, n=None):
  vals = [float(x) for x in str(s).split()]
  if n is not None and len(vals) < n:
    raise ValueError(f"expected {n} values, got '{s}'")
  return vals


def _merge_vec(default, given):
  """MJCF partial vectors keep the trailing default values (e.g. friction='.7')."""
  out = list(default)
  for i, v in enumerate(given[: len(out)]):
    out[i] = v
  return out


def quat_mul(a, b):
  return np.array(
    [
      a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3],
      a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2],
      a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1],
      a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0],
    ]
  )


def quat_to_mat(q):
  w, x, y, z = q
  return np.array(
    [
      [w * w + x * x - y * y - z * z, 2 * (x * y - w * z), 2 * (x * z + w * y)],
      [2 * (x * y + w * z), w * w - x * x + y * y - z * z, 2 * (y * z - w * x)],
      [2 * (x * z - w * y), 2 * (y * z + w * x), w * w - x * x - y * y + z * z],
    ]
  )


def mat_to_quat(R):
  """Rotation matrix -> unit quaternion (w first, w >= 0)."""
  tr = R[0, 0] + R[1, 1] + R[2, 2]
  if tr > 0:
    s = math.sqrt(tr + 1.0) * 2
    q = [0.25 * s, (R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s]
  elif R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]:
    s = math.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2]) * 2
    q = [(R[2, 1] - R[1, 2]) / s, 0.25 * s, (R[0, 1] + R[1, 0]) / s, (R[0, 2] + R[2, 0]) / s]
  elif R[1, 1] > R[2, 2]:
    s = math.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2]) * 2
    q = [(R[0, 2] - R[2, 0]) / s, (R[0, 1] + R[1, 0]) / s, 0.25 * s, (R[1, 2] + R[2, 1]) / s]
  else:
    s = math.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1]) * 2
    q = [(R[1, 0] - R[0, 1]) / s, (R[0, 2] + R[2, 0]) / s, (R[1, 2] + R[2, 1]) / s, 0.25 * s]
  q = np.array(q)
  if q[0] < 0:
    q = -q
  return q / np.linalg.norm(q)


def z2quat(vec):
  """Minimal rotation taking +z to `vec` (MuJoCo mjuu_z2quat convention)."""
  v = np.asarray(vec, dtype=float)
  n = np.linalg.norm(v)
  if n < MJ_MINVAL:
    return np.array([1.0, 0, 0, 0])
  v = v / n
  axis = np.cross([0.0, 0.0, 1.0], v)
  s = np.linalg.norm(axis)
  if s < 1e-10:
    if v[2] < 0:
      return np.array([0.0, 1.0, 0.0, 0.0])
    return np.array([1.0, 0, 0, 0])
  axis = axis / s
  ang = math.atan2(s, v[2])
  return np.array([math.cos(ang / 2), *(axis * math.sin(ang / 2))])


def rot_vec(q, v):
  return quat_to_mat(q) @ np.asarray(v, dtype=float)


class MjOption:
  def __init__(self):
    self.timestep = 0.002
    self.impratio = 1.0
    self.tolerance = 1e-8
    self.ls_tolerance = 0.01
    self.noslip_tolerance = 1e-6
    self.ccd_tolerance = 1e-6
    self.gravity = np.array([0.0, 0.0, -9.81])
    self.wind = np.zeros(3)
    self.magnetic = np.array([0.0, -0.5, 0.0])
    self.density = 0.0
    self.viscosity = 0.0
    self.o_margin = 0.0
    self.o_solref = np.array([0.02, 1.0])
    self.o_solimp = np.array([0.9, 0.95, 0.001, 0.5, 2.0])
    self.o_friction = np.array([1.0, 1.0, 0.005, 0.0001, 0.0001])
    self.integrator = int(IntegratorType.EULER)
    self.cone = int(ConeType.PYRAMIDAL)
    self.jacobian = int(JacobianType.AUTO)
    self.solver = int(SolverType.NEWTON)
    self.iterations = 100
    self.ls_iterations = 50
    self.noslip_iterations = 0
    self.ls_parallel = False  # Warp-only option from <custom><numeric name="ls_parallel" data="1"/>
    self.contact_sensor_maxmatch = 64  # Warp-only option (io.py:195-199), <custom><numeric>
    self.ccd_iterations = 35
    self.disableflags = 0
    self.enableflags = 0


class MjStatistic:
  def __init__(self):
    self.meaninertia = 1.0
    self.meanmass = 1.0
    self.meansize = 1.0
    self.extent = 1.0
    self.center = np.zeros(3)


class MjModel:
  """Host model with MuJoCo `mjModel` field names (subset used by the stepper)."""

  def __init__(self):
    self.opt = MjOption()
    self.stat = MjStatistic()

  def __repr__(self):
    return f"MjModel(nq={self.nq}, nv={self.nv}, nu={self.nu}, nbody={self.nbody}, ngeom={self.ngeom})"


class MjData:
  """Host state container mirroring the `mujoco.MjData` fields consumed by put_data."""

  def __init__(self, m: MjModel):
    self.time = 0.0
    self.qpos = m.qpos0.copy()
    self.qvel = np.zeros(m.nv)
    self.act = np.zeros(m.na)
    self.qacc_warmstart = np.zeros(m.nv)
    self.ctrl = np.zeros(m.nu)
    self.qfrc_applied = np.zeros(m.nv)
    self.xfrc_applied = np.zeros((m.nbody, 6))
    self.mocap_pos = np.zeros((m.nmocap, 3))
    self.mocap_quat = np.tile([1.0, 0, 0, 0], (m.nmocap, 1))
    self.eq_active = m.eq_active0.copy() if m.neq else np.zeros(0, dtype=np.uint8)
    self.qacc = np.zeros(m.nv)
    self.act_dot = np.zeros(m.na)
    self.ncon = 0
    self.nefc = 0
    self.solver_niter = np.zeros(1, dtype=int)
    for i, bid in enumerate(np.nonzero(m.body_mocapid >= 0)[0]):
      self.mocap_pos[m.body_mocapid[bid]] = m.body_pos[bid]
      self.mocap_quat[m.body_mocapid[bid]] = m.body_quat[bid]


def reset_data_keyframe(m: MjModel, d: MjData, key: int):
  """mj_resetDataKeyframe for the fields the stepper consumes."""
  fresh = MjData(m)
  d.__dict__.update(fresh.__dict__)
  d.time = float(m.key_time[key])
  d.qpos[:] = m.key_qpos[key]
  d.qvel[:] = m.key_qvel[key]
  if m.na:
    d.act[:] = m.key_act[key]
  if m.nu:
    d.ctrl[:] = m.key_ctrl[key]
  if m.nmocap:
    d.mocap_pos[:] = m.key_mpos[key].reshape(-1, 3)
    d.mocap_quat[:] = m.key_mquat[key].reshape(-1, 4)


# ---------------------------------------------------------------------------------------------
# parsing
# ---------------------------------------------------------------------------------------------


class _Default:
  def __init__(self, name, parent=None):
    self.name = name
    self.attrs = {k: dict(v) for k, v in (parent.attrs.items() if parent else [])}

  def get(self, kind):
    return self.attrs.setdefault(kind, {})


class _Body:
  def __init__(self, name, parent, childclass):
    self.name = name
    self.parent = parent
    self.childclass = childclass
    self.pos = np.zeros(3)
    self.quat = np.array([1.0, 0, 0, 0])
    self.inertial = None
    self.mocap = False
    self.gravcomp = 0.0
    self.joints = []
    self.geoms = []
    self.sites = []
    self.cams = []
    self.lights = []
    self.children = []


def _orientation(attrs, angle_scale, eulerseq="xyz"):
  """Frame orientation from quat / axisangle / euler / xyaxes / zaxis attributes."""
  if "quat" in attrs:
    q = np.array(_floats(attrs["quat"], 4))
    return q / np.linalg.norm(q)
  if "axisangle" in attrs:
    v = _floats(attrs["axisangle"], 4)
    axis = np.array(v[:3]) / np.linalg.norm(v[:3])
    ang = v[3] * angle_scale
    return np.array([math.cos(ang / 2), *(axis * math.sin(ang / 2))])
  if "euler" in attrs:
    e = np.array(_floats(attrs["euler"], 3)) * angle_scale
    q = np.array([1.0, 0, 0, 0])
    for i, ax in enumerate(eulerseq):
      axis = {"x": [1, 0, 0], "y": [0, 1, 0], "z": [0, 0, 1], "X": [1, 0, 0], "Y": [0, 1, 0], "Z": [0, 0, 1]}[ax]
      r = np.array([math.cos(e[i] / 2), *(np.array(axis) * math.sin(e[i] / 2))])
      q = quat_mul(q, r) if ax.islower() else quat_mul(r, q)
    return q / np.linalg.norm(q)
  if "xyaxes" in attrs:
    v = _floats(attrs["xyaxes"], 6)
    x = np.array(v[:3]) / np.linalg.norm(v[:3])
    y = np.array(v[3:6])
    y = y - x * np.dot(x, y)
    y = y / np.linalg.norm(y)
    z = np.cross(x, y)
    return mat_to_quat(np.stack([x, y, z], axis=1))
  if "zaxis" in attrs:
    return z2quat(_floats(attrs["zaxis"], 3))
  return None


class _Compiler:
  def __init__(self, root: ET.Element, basedir: str):
    self.root = root
    self.basedir = basedir
    self.angle_scale = math.pi / 180.0
    self.eulerseq = "xyz"
    self.autolimits = True
    self.inertiafromgeom = "auto"
    self.meshdir = ""
    self.boundmass = 0.0
    self.boundinertia = 0.0
    self.defaults = {}
    self.flexcomps = []
    self.m = MjModel()

  # -- defaults ------------------------------------------------------------------------------
  def _parse_default(self, elem, parent):
    name = elem.get("class", "main")
    d = _Default(name, parent)
    for child in elem:
      if child.tag == "default":
        continue
      kind = "actuator" if child.tag in _ACTUATOR_TAGS else child.tag
      attrs = d.get(kind)
      attrs.update(child.attrib)
      if kind == "actuator":
        attrs["__tag__"] = child.tag
    self.defaults[name] = d
    for child in elem:
      if child.tag == "default":
        self._parse_default(child, d)

  def _resolve(self, kind, elem, childclass):
    cls = elem.get("class", childclass or "main")
    d = self.defaults.get(cls)
    if d is None:
      raise ValueError(f"unknown default class '{cls}'")
    out = dict(d.attrs.get(kind, {}))
    out.update(elem.attrib)
    return out

  # -- tree ----------------------------------------------------------------------------------
  def _parse_body(self, elem, parent, childclass):
    if elem.tag == "worldbody":
      body = _Body("world", None, None)
    else:
      childclass = elem.get("childclass", childclass)
      body = _Body(elem.get("name", ""), parent, childclass)
      body.pos = np.array(_floats(elem.get("pos", "0 0 0"), 3))
      q = _orientation(elem.attrib, self.angle_scale, self.eulerseq)
      if q is not None:
        body.quat = q
      body.mocap = elem.get("mocap", "false") == "true"
      body.gravcomp = float(elem.get("gravcomp", 0.0))
    for child in elem:
      tag = child.tag
      if tag == "body":
        body.children.append(self._parse_body(child, body, childclass))
      elif tag == "joint":
        body.joints.append(self._resolve("joint", child, childclass))
      elif tag == "freejoint":
        a = {"type": "free", "name": child.get("name", "")}
        body.joints.append(a)
      elif tag == "geom":
        body.geoms.append(self._resolve("geom", child, childclass))
      elif tag == "site":
        body.sites.append(self._resolve("site", child, childclass))
      elif tag == "camera":
        body.cams.append(self._resolve("camera", child, childclass))
      elif tag == "light":
        body.lights.append(self._resolve("light", child, childclass))
      elif tag == "inertial":
        body.inertial = dict(child.attrib)
      elif tag == "frame":
        for sub in self._flatten_frame(child):
          self._parse_frame_child(sub, body, childclass)
      elif tag == "flexcomp":
        self._flexcomp(child, body, childclass)
    return body

  def _flexcomp(self, el, parent, childclass):
    """<flexcomp type="grid" | "direct" dim="1" | "2" | "3">: one body per vertex, each a child of
    `parent` at the vertex position with three slide joints (x, y, z) -- MuJoCo's flexcomp dof="full"
    -- and the vertex mass mass/npoint; <pin id="..."/> vertices get no joints (static).  Elements,
    edges, flaps, shells and the elasticity constants are built after the body tree is indexed
    (`_build_flex`).  Grid ordering: point (ix, iy, iz) has index (ix*cy + iy)*cz + iz and sits at
    spacing * (i - (count-1)/2); dim 1 links consecutive points of its one long axis, dim 2 splits each
    cell into two triangles, dim 3 each cube into six tetrahedra around its main diagonal (MuJoCo
    user_flexcomp.cc, restated: parity unpinned, no MuJoCo here)."""
    a = el.attrib
    ftype = a.get("type", "grid")
    if ftype not in ("grid", "direct"):
      raise NotImplementedError(f"flexcomp type '{ftype}' is not supported (grid and direct only)")
    dim = int(a.get("dim", 2))
    if dim not in (1, 2, 3):
      raise ValueError(f"flexcomp dim must be 1, 2 or 3, got {dim}")
    if a.get("dof", "full") != "full":
      raise NotImplementedError("only flexcomp dof='full' is supported")
    pos = np.array(_floats(a.get("pos", "0 0 0"), 3))
    q = _orientation(a, self.angle_scale, self.eulerseq)
    R = quat_to_mat(np.array([1.0, 0, 0, 0]) if q is None else np.asarray(q, dtype=float))
    name = a.get("name", f"flex{len(self.flexcomps)}")
    mass = float(a.get("mass", 1.0))
    pts, elems = [], []
    if ftype == "direct":
      # type="direct": the points (flexcomp frame) and the triangles (vertex index triples) as given
      loc = np.array(_floats(a["point"]), dtype=float).reshape(-1, 3)
      pts = [R @ p_ + pos for p_ in loc]
      tri = np.array([int(x) for x in a["element"].split()], dtype=np.int64).reshape(-1, dim + 1)
      if tri.size and (tri.min() < 0 or tri.max() >= len(pts)):
        raise ValueError(f"flexcomp '{name}': element index out of range")
      elems = [tuple(int(v) for v in t) for t in tri]
      npnt = len(pts)
    else:
      count = [int(x) for x in _floats(a.get("count", "10 10 1"), 3)]
      if dim == 1 and sum(c > 1 for c in count) != 1:
        raise NotImplementedError("dim=1 grid needs exactly one count > 1")
      if dim == 2 and count[2] != 1:
        raise NotImplementedError("dim=2 grid needs count[2] == 1")
      if dim == 3 and min(count) < 2:
        raise NotImplementedError("dim=3 grid needs every count >= 2")
      spacing = np.array(_floats(a.get("spacing", "0.02 0.02 0.02"), 3))
      npnt = count[0] * count[1] * count[2]
      for ix in range(count[0]):
        for iy in range(count[1]):
          for iz in range(count[2]):
            loc = spacing * (np.array([ix, iy, iz]) - 0.5 * (np.array(count) - 1))
            pts.append(R @ loc + pos)
      cy, cz = count[1], count[2]
      if dim == 1:
        elems = [(i, i + 1) for i in range(npnt - 1)]
      elif dim == 2:
        for ix in range(count[0] - 1):
          for iy in range(count[1] - 1):
            v00, v10, v11, v01 = ix * cy + iy, (ix + 1) * cy + iy, (ix + 1) * cy + iy + 1, ix * cy + iy + 1
            elems += [(v00, v10, v11), (v00, v11, v01)]
      else:
        idx = lambda i, j, k: (i * cy + j) * cz + k  # noqa: E731
        for ix in range(count[0] - 1):
          for iy in range(count[1] - 1):
            for iz in range(count[2] - 1):
              c = [idx(ix + (q & 1), iy + ((q >> 1) & 1), iz + ((q >> 2) & 1)) for q in range(8)]
              # Kuhn split: the six monotone paths 0 -> 7 through the cube (conforming across cells)
              for p1, p2 in ((1, 3), (1, 5), (2, 3), (2, 6), (4, 5), (4, 6)):
                t = [c[0], c[p1], c[p2], c[7]]
                X = np.array([pts[v] for v in t])
                if np.linalg.det(np.stack([X[1] - X[0], X[2] - X[0], X[3] - X[0]])) < 0:
                  t[1], t[2] = t[2], t[1]  # positive orientation
                elems.append(tuple(t))
    pinned = set()
    for pin in el.findall("pin"):
      pinned |= {int(v) for v in pin.get("id", "").split()}
    nfree = max(npnt - len(pinned), 1)
    bodies = []
    for i, p in enumerate(pts):
      b = _Body(f"{name}_{i}", parent, childclass)
      b.pos = np.asarray(p, dtype=float)
      if i in pinned:
        # a pinned vertex is a static body at its rest position (no dofs, no mass)
        b.inertial = {"pos": "0 0 0", "mass": "0", "diaginertia": "0 0 0"}
      else:
        b.inertial = {"pos": "0 0 0", "mass": repr(mass / nfree), "diaginertia": "0 0 0"}
        for ax in ("1 0 0", "0 1 0", "0 0 1"):
          b.joints.append({"type": "slide", "axis": ax, "name": f"{name}_{i}_{'xyz'[len(b.joints)]}"})
      parent.children.append(b)
      bodies.append(b)
    self.flexcomps.append(self._flex_params(el, name, dim, bodies, elems))

  def _flex_params(self, el, name, dim, bodies, elems):
    """The flex record of a <flexcomp> or an explicit <flex>: vertex bodies, elements and the
    <edge> / <elasticity> / <contact> children's parameters (MuJoCo's defaults)."""
    a = el.attrib
    edge = el.find("edge")
    elast = el.find("elasticity")
    contact = el.find("contact")
    ea = edge.attrib if edge is not None else {}
    la = elast.attrib if elast is not None else {}
    ca = contact.attrib if contact is not None else {}
    return dict(
      name=name, dim=dim, bodies=bodies, elems=np.array(elems, dtype=np.int32).reshape(-1, dim + 1),
      radius=float(a.get("radius", 0.005)),
      edge_equality=ea.get("equality", "false") == "true",
      edge_solref=_merge_vec([0.02, 1.0], _floats(ea.get("solref", "0.02 1"))),
      edge_solimp=_merge_vec([0.9, 0.95, 0.001, 0.5, 2.0], _floats(ea.get("solimp", "0.9 0.95 0.001 0.5 2"))),
      young=float(la.get("young", 0.0)), poisson=float(la.get("poisson", 0.0)),
      thickness=float(la.get("thickness", -1.0)), damping=float(la.get("damping", 0.0)),
      elastic2d={"none": 0, "bend": 1, "stretch": 2, "both": 3}[la.get("elastic2d", "none")],
      contype=int(ca.get("contype", 1)), conaffinity=int(ca.get("conaffinity", 1)), condim=int(ca.get("condim", 3)),
      friction=_merge_vec([1.0, 0.005, 0.0001], _floats(ca.get("friction", "1 0.005 0.0001"))),
      solref=_merge_vec([0.02, 1.0], _floats(ca.get("solref", "0.02 1"))),
      solimp=_merge_vec([0.9, 0.95, 0.001, 0.5, 2.0], _floats(ca.get("solimp", "0.9 0.95 0.001 0.5 2"))),
      margin=float(ca.get("margin", 0.0)), gap=float(ca.get("gap", 0.0)),
    )

  def _deformable(self, root):
    """<deformable><flex dim body="b0 b1 ..." element="..."/>: an explicit flex over existing bodies,
    one vertex per listed body at the body's origin (MuJoCo's <flex> without `vertex`); its elements,
    edges and elasticity are built like a flexcomp's (`_build_flex`)."""
    by_name = {b.name: b for b in self.bodies}
    for dfm in root.findall("deformable"):
      for el in dfm:
        if el.tag == "skin":
          continue
        if el.tag != "flex":
          raise NotImplementedError(f"<deformable><{el.tag}> is not supported")
        a = el.attrib
        dim = int(a.get("dim", 2))
        if dim not in (1, 2, 3):
          raise ValueError(f"flex dim must be 1, 2 or 3, got {dim}")
        if a.get("vertex", "").strip():
          raise NotImplementedError("<flex vertex=...> (vertices in body-local coordinates) is not supported; list one body per vertex")
        names = a.get("body", "").split()
        missing = [n for n in names if n not in by_name]
        if missing:
          raise ValueError(f"flex '{a.get('name', '')}': unknown bodies {missing}")
        elems = np.array([int(x) for x in a.get("element", "").split()], dtype=np.int64).reshape(-1, dim + 1)
        if elems.size and (elems.min() < 0 or elems.max() >= len(names)):
          raise ValueError(f"flex '{a.get('name', '')}': element index out of range")
        name = a.get("name", f"flex{len(self.flexcomps)}")
        self.flexcomps.append(self._flex_params(el, name, dim, [by_name[n] for n in names], [tuple(int(v) for v in t) for t in elems]))

  def _parse_frame_child(self, child, body, childclass):
    """A child of a <frame> whose pose has already been composed with the frame's."""
    tag = child.tag
    if tag == "body":
      body.children.append(self._parse_body(child, body, childclass))
    elif tag == "joint":
      body.joints.append(self._resolve("joint", child, childclass))
    elif tag == "geom":
      body.geoms.append(self._resolve("geom", child, childclass))
    elif tag == "site":
      body.sites.append(self._resolve("site", child, childclass))
    elif tag == "camera":
      body.cams.append(self._resolve("camera", child, childclass))
    elif tag == "light":
      body.lights.append(self._resolve("light", child, childclass))

  def _flatten_frame(self, frame):
    """<frame pos quat/euler/...>: compose the frame transform into each child (MJCF frame semantics)."""
    # childclass: the frame's children (and, for bodies, their subtrees) default to it unless they name a
    # class (bodies: a childclass) of their own; an inner frame's childclass was applied first
    fcls = frame.get("childclass")
    fpos = np.array(_floats(frame.get("pos", "0 0 0"), 3))
    fq = _orientation(frame.attrib, self.angle_scale, self.eulerseq)
    fq = np.array([1.0, 0, 0, 0]) if fq is None else np.asarray(fq, dtype=float)
    R = quat_to_mat(fq)
    out = []
    for child in list(frame):
      if child.tag == "frame":
        subs = self._flatten_frame(child)
      else:
        subs = [child]
      for c in subs:
        c = copy.deepcopy(c)
        a = c.attrib
        if fcls is not None:
          key = "childclass" if c.tag == "body" else "class"
          if key not in a:
            a[key] = fcls
        if c.tag == "geom" and "fromto" in a:
          ft = np.array(_floats(a["fromto"], 6))
          p0, p1 = R @ ft[:3] + fpos, R @ ft[3:] + fpos
          a["fromto"] = " ".join(repr(float(x)) for x in np.concatenate([p0, p1]))
        elif c.tag in ("body", "geom", "site", "camera", "light", "joint"):
          pos = np.array(_floats(a.get("pos", "0 0 0"), 3))
          a["pos"] = " ".join(repr(float(x)) for x in (R @ pos + fpos))
          if c.tag == "joint":
            if "axis" in a:
              a["axis"] = " ".join(repr(float(x)) for x in (R @ np.array(_floats(a["axis"], 3))))
          elif c.tag == "light" and "dir" in a:
            a["dir"] = " ".join(repr(float(x)) for x in (R @ np.array(_floats(a["dir"], 3))))
          else:
            q = _orientation(a, self.angle_scale, self.eulerseq)
            q = np.array([1.0, 0, 0, 0]) if q is None else np.asarray(q, dtype=float)
            for k in ("quat", "euler", "axisangle", "xyaxes", "zaxis"):
              a.pop(k, None)
            a["quat"] = " ".join(repr(float(x)) for x in quat_mul(fq, q))
        out.append(c)
    return out

  def _include(self, root):
    """Inline <include file=...> elements (recursive)."""
    for parent in list(root.iter()):
      for i, child in enumerate(list(parent)):
        if child.tag == "include":
          path = os.path.join(self.basedir, child.get("file"))
          sub = ET.parse(path).getroot()
          self._include(sub)
          parent.remove(child)
          for j, c in enumerate(list(sub)):
            parent.insert(i + j, c)

  # -- main ----------------------------------------------------------------------------------
  def compile(self) -> MjModel:
    root = self.root
    self._include(root)
    m = self.m
    m.model_name = root.get("model", "MuJoCo Model")

    comp = root.find("compiler")
    if comp is not None:
      if comp.get("angle", "degree") == "radian":
        self.angle_scale = 1.0
      self.eulerseq = comp.get("eulerseq", "xyz")
      self.autolimits = comp.get("autolimits", "true") == "true"
      self.inertiafromgeom = comp.get("inertiafromgeom", "auto")
      self.meshdir = comp.get("meshdir", "")
      self.boundmass = float(comp.get("boundmass", 0.0))
      self.boundinertia = float(comp.get("boundinertia", 0.0))

    for opt in root.findall("option"):
      self._parse_option(opt)
    # <custom><numeric>: the reference's Warp-only options (io.py:188-199): ls_parallel = 1 selects the
    # parallel linesearch, contact_sensor_maxmatch sizes the contact sensor's match list
    m.numeric = {}
    for cust in root.findall("custom"):
      for num in cust.findall("numeric"):
        m.numeric[num.get("name", "")] = _floats(num.get("data", "0"))
    if "ls_parallel" in m.numeric:
      m.opt.ls_parallel = m.numeric["ls_parallel"][0] == 1
    if "contact_sensor_maxmatch" in m.numeric:
      m.opt.contact_sensor_maxmatch = int(m.numeric["contact_sensor_maxmatch"][0])

    # defaults (top-level <default> is class 'main')
    top = _Default("main")
    self.defaults["main"] = top
    for dflt in root.findall("default"):
      for child in dflt:
        if child.tag == "default":
          self._parse_default(child, top)
        else:
          kind = "actuator" if child.tag in _ACTUATOR_TAGS else child.tag
          top.get(kind).update(child.attrib)
          if kind == "actuator":
            top.get(kind)["__tag__"] = child.tag

    world = _Body("world", None, None)
    for wb in root.findall("worldbody"):
      wbody = self._parse_body(wb, None, None)
      world.joints += wbody.joints
      world.geoms += wbody.geoms
      world.sites += wbody.sites
      world.cams += wbody.cams
      world.lights += wbody.lights
      for c in wbody.children:
        c.parent = world
        world.children.append(c)

    # DFS pre-order body list
    bodies = []

    def visit(b):
      bodies.append(b)
      for c in b.children:
        visit(c)

    visit(world)
    self.bodies = bodies
    self._deformable(root)
    self._build_tables(root)
    return m

  def _parse_option(self, opt):
    o = self.m.opt
    a = opt.attrib
    for k in ("timestep", "impratio", "tolerance", "ls_tolerance", "noslip_tolerance", "ccd_tolerance", "density", "viscosity", "o_margin"):
      if k in a:
        setattr(o, k, float(a[k]))
    for k in ("iterations", "ls_iterations", "noslip_iterations", "ccd_iterations"):
      if k in a:
        setattr(o, k, int(a[k]))
    for k in ("gravity", "wind", "magnetic"):
      if k in a:
        setattr(o, k, np.array(_floats(a[k], 3)))
    if "integrator" in a:
      o.integrator = int(_INTEGRATORS[a["integrator"].lower()])
    if "solver" in a:
      o.solver = int(_SOLVERS[a["solver"].lower()])
    if "cone" in a:
      o.cone = int(_CONES[a["cone"].lower()])
    if "jacobian" in a:
      o.jacobian = int(_JACOBIANS[a["jacobian"].lower()])
    for flag in opt.findall("flag"):
      for k, v in flag.attrib.items():
        if k in _DISABLE_NAMES:
          if v == "disable":
            o.disableflags |= int(_DISABLE_NAMES[k])
          else:
            o.disableflags &= ~int(_DISABLE_NAMES[k])
        elif k in _ENABLE_NAMES:
          if v == "enable":
            o.enableflags |= int(_ENABLE_NAMES[k])
          else:
            o.enableflags &= ~int(_ENABLE_NAMES[k])

  # ---------------------------------------------------------------------------------------
  def _build_tables(self, root):
    m = self.m
    bodies = self.bodies
    nbody = len(bodies)
    bid = {id(b): i for i, b in enumerate(bodies)}
    m.nbody = nbody
    m.body_names = [b.name for b in bodies]
    m.body_parentid = np.array([bid[id(b.parent)] if b.parent is not None else 0 for b in bodies], dtype=np.int32)
    m.body_pos = np.array([b.pos for b in bodies])
    m.body_quat = np.array([b.quat for b in bodies])
    m.body_gravcomp = np.array([b.gravcomp for b in bodies])
    m.ngravcomp = int((m.body_gravcomp > 0.0).sum())  # bodies with gravity compensation (io.py:2218-2219)

    # mocap
    mocapid = -np.ones(nbody, dtype=np.int32)
    nmocap = 0
    for i, b in enumerate(bodies):
      if b.mocap:
        mocapid[i] = nmocap
        nmocap += 1
    m.body_mocapid = mocapid
    m.nmocap = nmocap

    # joints / dofs
    jnt_rows, dof_rows = [], []
    body_jntadr = -np.ones(nbody, dtype=np.int32)
    body_jntnum = np.zeros(nbody, dtype=np.int32)
    body_dofadr = -np.ones(nbody, dtype=np.int32)
    body_dofnum = np.zeros(nbody, dtype=np.int32)
    nq = 0
    for i, b in enumerate(bodies):
      if b.joints:
        body_jntadr[i] = len(jnt_rows)
      body_jntnum[i] = len(b.joints)
      ndof_b = 0
      for ja in b.joints:
        jtype = _JOINT_TYPES[ja.get("type", "hinge")]
        free = ja.get("type") == "free" and len(ja) <= 2  # <freejoint/>: no defaults
        get = (lambda k, d=None: ja.get(k, _JOINT_DEFAULTS.get(k) if d is None else d)) if not free else (lambda k, d=None: _JOINT_DEFAULTS.get(k) if d is None else d)
        row = dict(
          name=ja.get("name", ""),
          type=int(jtype),
          bodyid=i,
          qposadr=nq,
          dofadr=len(dof_rows),
          pos=np.array(_floats(get("pos")) if isinstance(get("pos"), str) else get("pos"), dtype=float),
          axis=np.array(_floats(get("axis")) if isinstance(get("axis"), str) else get("axis"), dtype=float),
        )
        nrm = np.linalg.norm(row["axis"])
        row["axis"] = row["axis"] / nrm if nrm > 0 else np.array([0.0, 0.0, 1.0])

        def fval(k):
          v = get(k)
          return float(v) if isinstance(v, str) else float(v)

        def vval(k, n):
          v = get(k)
          given = _floats(v) if isinstance(v, str) else list(v)
          return np.array(_merge_vec(_JOINT_DEFAULTS[k], given))[:n]

        ascale = self.angle_scale if jtype in (JointType.HINGE, JointType.BALL) else 1.0
        rng = get("range")
        rng = (np.array(_floats(rng), dtype=float) if isinstance(rng, str) else np.array(rng, dtype=float)) * ascale
        lim = get("limited")
        if lim == "auto":
          limited = bool(self.autolimits and ("range" in ja) and jtype != JointType.FREE)
        else:
          limited = lim == "true"
        afl = get("actuatorfrclimited")
        afr = get("actuatorfrcrange")
        afr = np.array(_floats(afr)) if isinstance(afr, str) else np.array(afr, dtype=float)
        if afl == "auto":
          afl = bool(self.autolimits and "actuatorfrcrange" in ja)
        else:
          afl = afl == "true"
        row.update(
          stiffness=fval("stiffness"),
          damping=fval("damping"),
          armature=fval("armature"),
          frictionloss=fval("frictionloss"),
          springref=fval("springref") * (self.angle_scale if jtype == JointType.HINGE else 1.0),
          ref=fval("ref") * (self.angle_scale if jtype == JointType.HINGE else 1.0),
          margin=fval("margin"),
          solref=vval("solreflimit", 2),
          solimp=vval("solimplimit", 5),
          solreffriction=vval("solreffriction", 2),
          solimpfriction=vval("solimpfriction", 5),
          limited=limited,
          range=rng,
          actfrclimited=afl,
          actfrcrange=afr,
          actgravcomp=get("actuatorgravcomp") == "true",
        )
        ndof = {JointType.FREE: 6, JointType.BALL: 3}.get(jtype, 1)
        nqj = {JointType.FREE: 7, JointType.BALL: 4}.get(jtype, 1)
        for k in range(ndof):
          dof_rows.append(dict(bodyid=i, jntid=len(jnt_rows), **{kk: row[kk] for kk in ("armature", "damping", "frictionloss", "solreffriction", "solimpfriction")}))
        ndof_b += ndof
        nq += nqj
        jnt_rows.append(row)
      if ndof_b:
        body_dofadr[i] = len(dof_rows) - ndof_b
      body_dofnum[i] = ndof_b

    njnt = len(jnt_rows)
    nv = len(dof_rows)
    m.njnt, m.nv, m.nq = njnt, nv, nq
    m.body_jntadr, m.body_jntnum, m.body_dofadr, m.body_dofnum = body_jntadr, body_jntnum, body_dofadr, body_dofnum
    m.jnt_names = [r["name"] for r in jnt_rows]
    m.jnt_type = np.array([r["type"] for r in jnt_rows], dtype=np.int32)
    m.jnt_bodyid = np.array([r["bodyid"] for r in jnt_rows], dtype=np.int32)
    m.jnt_qposadr = np.array([r["qposadr"] for r in jnt_rows], dtype=np.int32)
    m.jnt_dofadr = np.array([r["dofadr"] for r in jnt_rows], dtype=np.int32)
    m.jnt_pos = np.array([r["pos"] for r in jnt_rows]).reshape(njnt, 3)
    m.jnt_axis = np.array([r["axis"] for r in jnt_rows]).reshape(njnt, 3)
    m.jnt_stiffness = np.array([r["stiffness"] for r in jnt_rows])
    m.jnt_limited = np.array([r["limited"] for r in jnt_rows], dtype=bool)
    m.jnt_range = np.array([r["range"] for r in jnt_rows]).reshape(njnt, 2)
    m.jnt_margin = np.array([r["margin"] for r in jnt_rows])
    m.jnt_solref = np.array([r["solref"] for r in jnt_rows]).reshape(njnt, 2)
    m.jnt_solimp = np.array([r["solimp"] for r in jnt_rows]).reshape(njnt, 5)
    m.jnt_actfrclimited = np.array([r["actfrclimited"] for r in jnt_rows], dtype=bool)
    m.jnt_actfrcrange = np.array([r["actfrcrange"] for r in jnt_rows]).reshape(njnt, 2)
    m.jnt_actgravcomp = np.array([r["actgravcomp"] for r in jnt_rows], dtype=np.int32)

    m.dof_bodyid = np.array([r["bodyid"] for r in dof_rows], dtype=np.int32)
    m.dof_jntid = np.array([r["jntid"] for r in dof_rows], dtype=np.int32)
    m.dof_armature = np.array([r["armature"] for r in dof_rows])
    m.dof_damping = np.array([r["damping"] for r in dof_rows])
    m.dof_frictionloss = np.array([r["frictionloss"] for r in dof_rows])
    m.dof_solref = np.array([r["solreffriction"] for r in dof_rows]).reshape(nv, 2)
    m.dof_solimp = np.array([r["solimpfriction"] for r in dof_rows]).reshape(nv, 5)

    # qpos0 / qpos_spring
    qpos0 = np.zeros(nq)
    qpos_spring = np.zeros(nq)
    for j, r in enumerate(jnt_rows):
      a = r["qposadr"]
      if r["type"] == JointType.FREE:
        b = bodies[r["bodyid"]]
        qpos0[a : a + 3] = b.pos
        qpos0[a + 3 : a + 7] = b.quat
        qpos_spring[a : a + 7] = qpos0[a : a + 7]
      elif r["type"] == JointType.BALL:
        qpos0[a : a + 4] = [1, 0, 0, 0]
        qpos_spring[a : a + 4] = [1, 0, 0, 0]
      else:
        qpos0[a] = r["ref"]
        qpos_spring[a] = r["springref"]
    m.qpos0 = qpos0
    m.qpos_spring = qpos_spring

    # body tree arrays
    parent = m.body_parentid
    rootid = np.zeros(nbody, dtype=np.int32)
    weldid = np.zeros(nbody, dtype=np.int32)
    for i in range(1, nbody):
      rootid[i] = i if parent[i] == 0 else rootid[parent[i]]
      weldid[i] = i if body_jntnum[i] > 0 else weldid[parent[i]]
    m.body_rootid, m.body_weldid = rootid, weldid

    # dof_parentid: previous dof along the kinematic chain
    dof_parentid = -np.ones(nv, dtype=np.int32)
    for i in range(nbody):
      if body_dofnum[i] == 0:
        continue
      # last dof of nearest ancestor with dofs
      p = parent[i]
      prev = -1
      while p > 0:
        if body_dofnum[p] > 0:
          prev = body_dofadr[p] + body_dofnum[p] - 1
          break
        p = parent[p]
      for k in range(body_dofnum[i]):
        dof_parentid[body_dofadr[i] + k] = prev
        prev = body_dofadr[i] + k
    m.dof_parentid = dof_parentid

    # sparse M layout (MuJoCo dof_Madr: diagonal then ancestors)
    dof_Madr = np.zeros(nv, dtype=np.int32)
    nM = 0
    for i in range(nv):
      dof_Madr[i] = nM
      j = i
      while j >= 0:
        nM += 1
        j = dof_parentid[j]
    m.dof_Madr = dof_Madr
    m.nM = nM
    # CSR lower triangle (ancestors ascending, diagonal last) used by the sparse LDL
    M_rownnz = np.zeros(nv, dtype=np.int32)
    M_rowadr = np.zeros(nv, dtype=np.int32)
    colind, mapM2M = [], []
    for i in range(nv):
      anc = []
      j = i
      k = 0
      while j >= 0:
        anc.append((j, dof_Madr[i] + k))
        j = dof_parentid[j]
        k += 1
      anc = anc[::-1]
      M_rowadr[i] = len(colind)
      M_rownnz[i] = len(anc)
      for j, madr in anc:
        colind.append(j)
        mapM2M.append(madr)
    m.M_rownnz, m.M_rowadr = M_rownnz, M_rowadr
    m.M_colind = np.array(colind, dtype=np.int32)
    m.mapM2M = np.array(mapM2M, dtype=np.int32)
    m.nC = nM

    self._load_meshes(root)
    self._load_hfields(root)
    self._build_geoms()
    self._build_inertia()
    self._build_sites_cams_lights()
    self._build_tendons(root)
    self._build_actuators(root)
    self._build_contact(root)
    self._build_keys(root)
    self._build_flex()
    self._build_equality(root)
    self._build_sensors(root)
    m.body_subtreemass = self._subtreemass()
    set_const(m)

  # ---------------------------------------------------------------------------------------
  def _load_meshes(self, root):
    """<asset><mesh>: vertices of STL / OBJ files, scaled, repeated vertices removed in
    first-occurrence order (MuJoCo user_mesh.cc).  The vertices stay in the file's frame: MuJoCo also
    moves them to the mesh's inertial frame and folds that offset into geom_pos / geom_quat, which
    leaves the world-space geometry -- and so every contact -- unchanged; only the reported
    geom_xpos / geom_xmat of mesh geoms differ (parity unpinned: no MuJoCo here)."""
    m = self.m
    self.mesh_id = {}
    self.mesh_data = []  # (vertices (n, 3) float64, triangles (t, 3) int)
    for asset in root.findall("asset"):
      for me in asset.findall("mesh"):
        a = self._resolve("mesh", me, None)
        if "file" in a:
          v, f = _read_mesh_file(os.path.join(self.basedir, self.meshdir, a["file"]))
        elif "vertex" in a:  # inline mesh: vertices, faces given or the convex hull (MuJoCo user_mesh.cc)
          v = np.array(_floats(a["vertex"]), dtype=np.float64).reshape(-1, 3)
          f = np.array(_floats(a["face"]), dtype=np.int64).reshape(-1, 3) if "face" in a else _hull_faces(v)
        else:
          raise NotImplementedError("<mesh> needs a file or inline vertices")
        v = v * np.array(_merge_vec([1.0, 1.0, 1.0], _floats(a.get("scale", "1 1 1"))))
        _, first, inv = np.unique(v, axis=0, return_index=True, return_inverse=True)
        order = np.argsort(first)  # unique rows in first-occurrence order
        remap = np.empty(len(order), dtype=np.int64)
        remap[order] = np.arange(len(order))
        v = v[first[order]]
        f = remap[inv.reshape(-1)[f]]
        name = a.get("name") or os.path.splitext(os.path.basename(a.get("file", "")))[0]
        self.mesh_id[name] = len(self.mesh_data)
        self.mesh_data.append((v, f))
    m.nmesh = len(self.mesh_data)
    m.mesh_vertnum = np.array([len(v) for v, _ in self.mesh_data], dtype=np.int32)
    m.mesh_vertadr = np.concatenate([[0], np.cumsum(m.mesh_vertnum)[:-1]]).astype(np.int32) if m.nmesh else np.zeros(0, np.int32)
    m.mesh_vert = np.concatenate([v for v, _ in self.mesh_data]) if m.nmesh else np.zeros((0, 3))
    m.nmeshvert = int(m.mesh_vertnum.sum())
    # per-vertex normals (MuJoCo's mesh_normal without tangent frames: normalnum = vertnum): the
    # area-weighted mean of the adjacent triangles' normals, in the mesh frame (mesh_quat identity: this
    # compiler keeps mesh vertices in their file frame)
    normals = [_vertex_normals(v, f) for v, f in self.mesh_data]
    m.mesh_normal = np.concatenate(normals).reshape(-1, 3) if m.nmesh else np.zeros((0, 3))
    m.mesh_normaladr = m.mesh_vertadr.copy()
    m.mesh_normalnum = m.mesh_vertnum.copy()
    m.nmeshnormal = int(m.mesh_normalnum.sum())
    # polygon data of each mesh's convex hull (MuJoCo's mesh_poly* fields; multi-contact, collision_gjk.py:1403-1790)
    polys = [_mesh_polygons(v) for v, _ in self.mesh_data]
    m.mesh_polynum = np.array([len(p[0]) for p in polys], dtype=np.int32)
    m.mesh_polyadr = np.concatenate([[0], np.cumsum(m.mesh_polynum)[:-1]]).astype(np.int32) if m.nmesh else np.zeros(0, np.int32)
    m.mesh_polynormal = np.concatenate([p[1] for p in polys]).reshape(-1, 3) if m.nmesh else np.zeros((0, 3))
    loops = [lp for p in polys for lp in p[0]]
    m.mesh_polyvertnum = np.array([len(lp) for lp in loops], dtype=np.int32)
    m.mesh_polyvertadr = np.concatenate([[0], np.cumsum(m.mesh_polyvertnum)[:-1]]).astype(np.int32) if loops else np.zeros(0, np.int32)
    m.mesh_polyvert = np.array([i for lp in loops for i in lp], dtype=np.int32)
    pmaps = [mp for p in polys for mp in p[2]]  # per vertex (all meshes in order): its polygons
    m.mesh_polymapnum = np.array([len(mp) for mp in pmaps], dtype=np.int32)
    m.mesh_polymapadr = np.concatenate([[0], np.cumsum(m.mesh_polymapnum)[:-1]]).astype(np.int32) if pmaps else np.zeros(0, np.int32)
    m.mesh_polymap = np.array([i for mp in pmaps for i in mp], dtype=np.int32)
    m.nmeshpoly, m.nmeshpolyvert, m.nmeshpolymap = len(loops), len(m.mesh_polyvert), len(m.mesh_polymap)

  def _load_hfields(self, root):
    """<asset><hfield>: nrow x ncol elevation grid (row 0 at -y, MuJoCo's mjModel.hfield_data order), size =
    (x half-extent, y half-extent, top, base).  `elevation` values are normalised to [0, 1] by subtracting
    the minimum and dividing by the range when it is non-zero (MuJoCo user_hfield); without it the grid is
    flat.  A `file` gives the grid instead (_read_hfield_file: a PNG image or MuJoCo's binary format), its
    values normalised the same way.""" 
    m = self.m
    self.hfield_id = {}
    sizes, nrows, ncols, datas = [], [], [], []
    for asset in root.findall("asset"):
      for he in asset.findall("hfield"):
        a = self._resolve("hfield", he, None)
        fdata = None
        if "file" in a:
          nrow, ncol, fdata = _read_hfield_file(os.path.join(self.basedir, a.get("file")))
          a = dict(a, nrow=str(nrow), ncol=str(ncol))
        nrow, ncol = int(a.get("nrow", 0)), int(a.get("ncol", 0))
        if nrow < 2 or ncol < 2:
          raise ValueError("<hfield> needs nrow >= 2 and ncol >= 2")
        size = _floats(a.get("size", "0 0 0 0"), 4)
        if min(size) <= 0:
          raise ValueError("<hfield> size must be positive")
        if fdata is not None or "elevation" in a:
          e = fdata if fdata is not None else np.array(_floats(a["elevation"]), dtype=np.float64)
          if e.size != nrow * ncol:
            raise ValueError(f"<hfield> elevation has {e.size} values, nrow * ncol = {nrow * ncol}")
          lo, hi = e.min(), e.max()
          e = (e - lo) / (hi - lo) if hi > lo else e - lo
        else:
          e = np.zeros(nrow * ncol)
        self.hfield_id[a.get("name", "")] = len(sizes)
        sizes.append(size)
        nrows.append(nrow)
        ncols.append(ncol)
        datas.append(e)
    m.nhfield = len(sizes)
    m.hfield_size = np.array(sizes, dtype=np.float64).reshape(-1, 4)
    m.hfield_nrow = np.array(nrows, dtype=np.int32)
    m.hfield_ncol = np.array(ncols, dtype=np.int32)
    m.hfield_adr = np.concatenate([[0], np.cumsum(m.hfield_nrow * m.hfield_ncol)[:-1]]).astype(np.int32) if m.nhfield else np.zeros(0, np.int32)
    m.hfield_data = np.concatenate(datas) if datas else np.zeros(0)
    m.nhfielddata = int(m.hfield_data.size)

  def _build_flex(self):
    """mjModel flex_* tables of the flexcomps (MuJoCo user_flex.cc semantics, restated).

    Edges are numbered in first-encounter order over the elements, each element contributing its local
    edges in the order of passive.py:_flex_elasticity (:606-613): (0,1) for a segment; (1,2), (2,0),
    (0,1) for a triangle; (0,1), (1,2), (2,0), (2,3), (0,3), (1,3) for a tetrahedron.  flex_edgeflap
    holds the vertex opposite the edge in its first and second triangle (-1 on the boundary, and for
    dims 1 / 3).  flex_bending holds the 16 coefficients of the discrete quadratic bending energy of a
    triangle edge's two triangles (cotangent weights, Wardetzky et al. 2007 / Bergou et al. 2006)
    scaled by mu*thickness^3 / (8*(A0 + A1)) with mu = young / (2*(1+poisson)), and a zero 17th (flat
    rest shape).  flex_stiffness holds, per element, the upper triangle of the edge metric M of the
    Saint Venant-Kirchhoff energy in the squared-edge-length strains s_e = L_e^2 - L0_e^2 that
    passive.py:_flex_elasticity evaluates (energy = 1/4 s' M s; `_svk_metric`): volumetric for dim 3,
    the membrane (elastic2d stretch / both) for dim 2, axial for dim 1.  flex_shell lists the boundary
    triangles of a dim-3 flex (faces of one tetrahedron only, outward), the triangles
    collision_flex.py:531-683 collides.  These compiler constants are parity unpinned: MuJoCo's
    compiler is not available."""
    m = self.m
    bid = {id(b): i for i, b in enumerate(self.bodies)}
    fl = self.flexcomps
    m.nflex = len(fl)
    vertadr, vertnum, edgeadr, edgenum, elemadr, elemnum, elemdataadr, elemedgeadr = [], [], [], [], [], [], [], []
    vertbodyid, edges, flaps, elemdata, elemedge, bending, stiffness, length0, vertflexid = [], [], [], [], [], [], [], [], []
    shellnum, shelladr, shell = [], [], []
    nelem_tot = 0
    for f, fc in enumerate(fl):
      dim = fc["dim"]
      vb = [bid[id(b)] for b in fc["bodies"]]
      x = np.array([_body_world_pos(b) for b in fc["bodies"]])  # rest positions, world frame
      vertadr.append(len(vertbodyid))
      vertnum.append(len(vb))
      vertbodyid += vb
      vertflexid += [f] * len(vb)
      el = fc["elems"]
      ledges = _FLEX_LOCAL_EDGES[dim]
      elemadr.append(nelem_tot)
      elemnum.append(len(el))
      nelem_tot += len(el)
      elemdataadr.append(len(elemdata))
      elemedgeadr.append(len(elemedge))
      eid, fe, tri_of_edge = {}, [], []
      for t, tri in enumerate(el):
        for a_, b_ in ledges:
          key = (min(tri[a_], tri[b_]), max(tri[a_], tri[b_]))
          if key not in eid:
            eid[key] = len(fe)
            fe.append(key)
            tri_of_edge.append([])
          if dim == 2:
            tri_of_edge[eid[key]].append((t, 3 - a_ - b_))
          elemedge.append(eid[key])
        elemdata += [int(v) for v in tri]
      edgeadr.append(len(edges))
      edgenum.append(len(fe))
      young, poisson = fc["young"], fc["poisson"]
      mu = young / (2.0 * (1.0 + poisson))
      for e, (v0, v1) in enumerate(fe):
        edges.append((v0, v1))
        fp = [int(el[t][k]) for t, k in tri_of_edge[e]][:2] + [-1, -1]
        flaps.append((fp[0], fp[1]))
        length0.append(float(np.linalg.norm(x[v1] - x[v0])))
        coef = np.zeros(17)
        if dim == 2 and fc["elastic2d"] in (1, 3) and fp[1] >= 0 and fc["thickness"] > 0 and mu > 0:
          coef[:16] = _bending_coef(x[[v0, v1, fp[0], fp[1]]], mu, fc["thickness"])
        bending.append(coef)
      # element metrics: dim 3 always (young > 0), dim 2 with elastic2d stretch / both, dim 1 axial
      use = young > 0 and (dim != 2 or fc["elastic2d"] >= 2)
      if dim == 2 and use and not fc["thickness"] > 0:
        raise ValueError(f"flexcomp '{fc['name']}': membrane elasticity needs a positive thickness")
      for tri in el:
        coef = np.zeros(21)
        if use:
          M = _svk_metric(x[list(tri)], young, poisson, dim, fc["thickness"], fc["radius"])
          iu = np.triu_indices(len(ledges))
          coef[:len(iu[0])] = M[iu]
        stiffness.append(coef)
      # dim 3: boundary faces (faces of exactly one tetrahedron), oriented away from the fourth vertex
      shelladr.append(len(shell))
      ns = 0
      if dim == 3:
        faces = {}
        order = []
        for t, tet in enumerate(el):
          for skip in range(4):
            face = [int(tet[k]) for k in range(4) if k != skip]
            key = tuple(sorted(face))
            if key not in faces:
              faces[key] = [face, int(tet[skip]), 0]
              order.append(key)
            faces[key][2] += 1
        for key in order:
          face, opp, cnt = faces[key]
          if cnt != 1:
            continue
          a_, b_, c_ = face
          if np.dot(np.cross(x[b_] - x[a_], x[c_] - x[a_]), x[opp] - x[a_]) > 0:
            b_, c_ = c_, b_
          shell += [a_, b_, c_]
          ns += 1
      shellnum.append(ns)
    m.flex_dim = np.array([fc["dim"] for fc in fl], dtype=np.int32)
    m.flex_vertadr, m.flex_vertnum = np.array(vertadr, dtype=np.int32), np.array(vertnum, dtype=np.int32)
    m.flex_edgeadr, m.flex_edgenum = np.array(edgeadr, dtype=np.int32), np.array(edgenum, dtype=np.int32)
    m.flex_elemadr, m.flex_elemnum = np.array(elemadr, dtype=np.int32), np.array(elemnum, dtype=np.int32)
    m.flex_elemdataadr = np.array(elemdataadr, dtype=np.int32)
    m.flex_elemedgeadr = np.array(elemedgeadr, dtype=np.int32)
    m.nflexvert, m.nflexedge, m.nflexelem, m.nflexelemdata = len(vertbodyid), len(edges), nelem_tot, len(elemdata)
    m.nflexelemedge = len(elemedge)
    m.flex_vertbodyid = np.array(vertbodyid, dtype=np.int32)
    m.flex_vertflexid = np.array(vertflexid, dtype=np.int32)
    m.flex_vert = np.zeros((m.nflexvert, 3))
    m.flex_centered = np.ones(m.nflex, dtype=np.int32)
    m.flex_edge = np.array(edges, dtype=np.int32).reshape(-1, 2)
    m.flex_edgeflap = np.array(flaps, dtype=np.int32).reshape(-1, 2)
    m.flex_elem = np.array(elemdata, dtype=np.int32)
    m.flex_elemedge = np.array(elemedge, dtype=np.int32)
    m.flex_shellnum = np.array(shellnum, dtype=np.int32)
    m.flex_shelldataadr = np.array(shelladr, dtype=np.int32)
    m.flex_shell = np.array(shell, dtype=np.int32)
    m.nflexshelldata = len(shell)
    m.flexedge_length0 = np.array(length0)
    m.flex_bending = np.array(bending).reshape(-1, 17)
    m.flex_stiffness = np.array(stiffness).reshape(-1, 21)
    m.flex_damping = np.array([fc["damping"] for fc in fl])
    m.flex_radius = np.array([fc["radius"] for fc in fl])
    m.flex_margin = np.array([fc["margin"] for fc in fl])
    m.flex_gap = np.array([fc["gap"] for fc in fl])
    m.flex_condim = np.array([fc["condim"] for fc in fl], dtype=np.int32)
    m.flex_friction = np.array([fc["friction"] for fc in fl]).reshape(-1, 3)
    m.flex_solref = np.array([fc["solref"] for fc in fl]).reshape(-1, 2)
    m.flex_solimp = np.array([fc["solimp"] for fc in fl]).reshape(-1, 5)
    m.flex_contype = np.array([fc["contype"] for fc in fl], dtype=np.int32)
    m.flex_conaffinity = np.array([fc["conaffinity"] for fc in fl], dtype=np.int32)
    # flexedge_invweight0 = J M^-1 J' at qpos0 for the vertex-own-dof edge Jacobian (smooth.py:261-355):
    # each vertex body carries three orthogonal slide dofs and the vertex mass
    iw = []
    for f in range(m.nflex):
      for e in range(m.flex_edgenum[f]):
        vs = m.flex_edge[m.flex_edgeadr[f] + e] + m.flex_vertadr[f]
        bs = [m.flex_vertbodyid[v] for v in vs]
        iw.append(sum(1.0 / m.body_mass[b] for b in bs if m.body_dofnum[b]))
    m.flexedge_invweight0 = np.array(iw)

  def _build_geoms(self):
    m = self.m
    rows = []
    for i, b in enumerate(self.bodies):
      for ga in b.geoms:
        rows.append(self._geom(ga, i))
    ng = len(rows)
    m.ngeom = ng
    m.geom_names = [r["name"] for r in rows]
    m.geom_type = np.array([r["type"] for r in rows], dtype=np.int32)
    m.geom_bodyid = np.array([r["bodyid"] for r in rows], dtype=np.int32)
    m.geom_contype = np.array([r["contype"] for r in rows], dtype=np.int32)
    m.geom_conaffinity = np.array([r["conaffinity"] for r in rows], dtype=np.int32)
    m.geom_condim = np.array([r["condim"] for r in rows], dtype=np.int32)
    m.geom_priority = np.array([r["priority"] for r in rows], dtype=np.int32)
    m.geom_group = np.array([r["group"] for r in rows], dtype=np.int32)
    m.geom_size = np.array([r["size"] for r in rows]).reshape(ng, 3)
    m.geom_pos = np.array([r["pos"] for r in rows]).reshape(ng, 3)
    m.geom_quat = np.array([r["quat"] for r in rows]).reshape(ng, 4)
    m.geom_friction = np.array([r["friction"] for r in rows]).reshape(ng, 3)
    m.geom_solmix = np.array([r["solmix"] for r in rows])
    m.geom_solref = np.array([r["solref"] for r in rows]).reshape(ng, 2)
    m.geom_solimp = np.array([r["solimp"] for r in rows]).reshape(ng, 5)
    m.geom_margin = np.array([r["margin"] for r in rows])
    m.geom_gap = np.array([r["gap"] for r in rows])
    m.geom_rbound = np.array([r["rbound"] for r in rows])
    m.geom_aabb = np.array([r["aabb"] for r in rows]).reshape(ng, 6)
    m.geom_dataid = np.array([r["dataid"] for r in rows], dtype=np.int32)
    m.geom_fluid = np.array([r["fluid"] for r in rows]).reshape(ng, NFLUID)
    self.geom_mesh_props = [(r["mesh_com"], r["mesh_I"]) for r in rows]
    m.geom_mass_ = np.array([r["mass"] for r in rows])
    m.geom_inertia_ = np.array([r["inertia"] for r in rows]).reshape(ng, 3)
    m.geom_rgba = np.tile([0.5, 0.5, 0.5, 1.0], (ng, 1))
    body_geomadr = -np.ones(m.nbody, dtype=np.int32)
    body_geomnum = np.zeros(m.nbody, dtype=np.int32)
    for g, r in enumerate(rows):
      b = r["bodyid"]
      if body_geomnum[b] == 0:
        body_geomadr[b] = g
      body_geomnum[b] += 1
    m.body_geomadr, m.body_geomnum = body_geomadr, body_geomnum

  def _geom(self, ga, bodyid):
    gtype = _GEOM_TYPES[ga.get("type", _GEOM_DEFAULTS["type"])]
    if gtype == GeomType.SDF:
      raise NotImplementedError(f"geom type {gtype.name} not supported by the MJCF compiler")
    # heightfields may sit on moving bodies: the collision routines take the geom's frame; like planes they
    # contribute no mass (the body's other geoms or an explicit <inertial> give it one)
    # mesh geoms: the mesh file is not read (no mesh collision or mesh-derived inertia here), so
    # the geom keeps its declared frame; put_model rejects meshes that can collide and bodies
    # whose inertia would come from a mesh.

    def vec(k, n):
      given = _floats(ga[k]) if k in ga else []
      return np.array(_merge_vec(_GEOM_DEFAULTS[k], given))[:n]

    size = vec("size", 3)
    pos = np.array(_floats(ga.get("pos", "0 0 0"), 3))
    quat = _orientation(ga, self.angle_scale, self.eulerseq)
    quat = np.array([1.0, 0, 0, 0]) if quat is None else quat
    if "fromto" in ga:
      ft = np.array(_floats(ga["fromto"], 6))
      a, b = ft[:3], ft[3:]
      pos = 0.5 * (a + b)
      quat = z2quat(b - a)
      hl = 0.5 * np.linalg.norm(b - a)
      if gtype in (GeomType.CAPSULE, GeomType.CYLINDER):
        size[1] = hl
      elif gtype == GeomType.BOX:
        size[2] = hl
      elif gtype == GeomType.ELLIPSOID:
        size[2] = hl
    r = size[0]
    if gtype == GeomType.SPHERE:
      vol = 4.0 / 3.0 * math.pi * r**3
      rbound = r
      aabb = [0, 0, 0, r, r, r]
    elif gtype == GeomType.CAPSULE:
      vol = math.pi * r * r * 2 * size[1] + 4.0 / 3.0 * math.pi * r**3
      rbound = r + size[1]
      aabb = [0, 0, 0, r, r, size[1] + r]
    elif gtype == GeomType.CYLINDER:
      vol = math.pi * r * r * 2 * size[1]
      rbound = math.sqrt(r * r + size[1] ** 2)
      aabb = [0, 0, 0, r, r, size[1]]
    elif gtype == GeomType.BOX:
      vol = 8 * size[0] * size[1] * size[2]
      rbound = float(np.linalg.norm(size))
      aabb = [0, 0, 0, size[0], size[1], size[2]]
    elif gtype == GeomType.ELLIPSOID:
      vol = 4.0 / 3.0 * math.pi * size[0] * size[1] * size[2]
      rbound = float(np.max(size))
      aabb = [0, 0, 0, size[0], size[1], size[2]]
    elif gtype == GeomType.PLANE:
      vol = 0.0
      rbound = 0.0
      aabb = [0, 0, 0, size[0], size[1], 0.0]
    elif gtype == GeomType.HFIELD:
      if ga.get("hfield") not in self.hfield_id:
        raise ValueError(f"geom {ga.get('name', '')}: unknown hfield '{ga.get('hfield')}'")
      dataid = self.hfield_id[ga["hfield"]]
      hs = self.m.hfield_size[dataid]
      vol = 0.0
      size = np.array([hs[0], hs[1], 0.5 * (hs[2] + hs[3])])
      rbound = float(math.sqrt(hs[0] ** 2 + hs[1] ** 2 + max(hs[2], hs[3]) ** 2))
      aabb = [0, 0, 0.5 * (hs[2] - hs[3]), hs[0], hs[1], 0.5 * (hs[2] + hs[3])]
    elif gtype == GeomType.MESH:
      if ga.get("mesh") not in self.mesh_id:
        raise ValueError(f"geom {ga.get('name', '')}: unknown mesh '{ga.get('mesh')}'")
      dataid = self.mesh_id[ga["mesh"]]
      mv, mf = self.mesh_data[dataid]
      vol, mesh_com, mesh_I1 = _mesh_mass_props(mv, mf)
      rbound = float(np.sqrt((mv * mv).sum(axis=1).max()))
      lo, hi = mv.min(axis=0), mv.max(axis=0)
      aabb = list(0.5 * (lo + hi)) + list(0.5 * (hi - lo))
      size = 0.5 * (hi - lo)
    else:
      raise NotImplementedError(gtype)
    density = float(ga.get("density", _GEOM_DEFAULTS["density"]))
    mass = float(ga["mass"]) if "mass" in ga else density * vol
    fluid = _geom_fluid(ga, gtype, size)
    if gtype == GeomType.MESH:
      inertia = np.zeros(3)
      # full inertia about the mesh COM in the geom frame (unit-density integrals scaled to mass)
      mesh_I = mesh_I1 * (mass / vol) if vol > MJ_MINVAL else np.zeros((3, 3))
    else:
      inertia = _geom_inertia(gtype, size, mass)
    return dict(
      name=ga.get("name", ""),
      type=int(gtype),
      bodyid=bodyid,
      contype=int(ga.get("contype", 1)),
      conaffinity=int(ga.get("conaffinity", 1)),
      condim=int(ga.get("condim", 3)),
      priority=int(ga.get("priority", 0)),
      group=int(ga.get("group", 0)),
      size=size,
      pos=pos,
      quat=quat,
      friction=vec("friction", 3),
      solmix=float(ga.get("solmix", 1.0)),
      solref=vec("solref", 2),
      solimp=vec("solimp", 5),
      margin=float(ga.get("margin", 0.0)),
      gap=float(ga.get("gap", 0.0)),
      rbound=rbound,
      aabb=aabb,
      mass=mass if gtype not in (GeomType.PLANE, GeomType.HFIELD) else 0.0,
      inertia=inertia,
      dataid=dataid if gtype in (GeomType.MESH, GeomType.HFIELD) else -1,
      fluid=fluid,
      mesh_com=mesh_com if gtype == GeomType.MESH else None,
      mesh_I=mesh_I if gtype == GeomType.MESH else None,
    )

  def _build_inertia(self):
    """Body inertial frames from <inertial> or from geoms (MuJoCo inertiafromgeom='auto')."""
    m = self.m
    nb = m.nbody
    m.body_mass = np.zeros(nb)
    m.body_ipos = np.zeros((nb, 3))
    m.body_iquat = np.tile([1.0, 0, 0, 0], (nb, 1))
    m.body_inertia = np.zeros((nb, 3))
    for i, b in enumerate(self.bodies):
      if i == 0:
        continue
      if b.inertial is not None and self.inertiafromgeom != "true":
        ia = b.inertial
        m.body_mass[i] = float(ia["mass"])
        m.body_ipos[i] = _floats(ia.get("pos", "0 0 0"), 3)
        if "fullinertia" in ia:
          f = _floats(ia["fullinertia"], 6)
          I = np.array([[f[0], f[3], f[4]], [f[3], f[1], f[5]], [f[4], f[5], f[2]]])
          w, V = _eig3(I)
          iq = mat_to_quat(V)
          m.body_iquat[i] = quat_mul(np.array([1.0, 0, 0, 0]), iq)
          m.body_inertia[i] = w
        else:
          q = _orientation(ia, self.angle_scale, self.eulerseq)
          m.body_iquat[i] = q if q is not None else [1, 0, 0, 0]
          m.body_inertia[i] = _floats(ia["diaginertia"], 3)
        continue
      # a heightfield geom's mass and inertia (MuJoCo's compiler prices it like a box from the heightfield
      # asset) are not reproduced: a moving body with one needs an explicit <inertial> (parity unpinned
      # otherwise; static bodies never use their inertia)
      if m.body_weldid[i] != 0 and any(m.geom_bodyid[g] == i and m.geom_type[g] == GeomType.HFIELD for g in range(m.ngeom)):
        raise NotImplementedError(f"body {i}: a heightfield geom on a moving body needs an explicit <inertial> (its "
                                  "geom-derived mass / inertia is not built)")
      # massless geoms (e.g. density="0" visual meshes) do not shape the inertial frame
      geoms = [g for g in range(m.ngeom) if m.geom_bodyid[g] == i and m.geom_type[g] != GeomType.PLANE and m.geom_mass_[g] > 0]
      if not geoms:
        continue
      mass = sum(m.geom_mass_[g] for g in geoms)
      if mass < MJ_MINVAL:
        continue
      # per geom: COM and inertia about it, in the body frame (meshes: COM offset + full tensor)
      gcom, gI = {}, {}
      for g in geoms:
        R = quat_to_mat(m.geom_quat[g])
        mc, mI = self.geom_mesh_props[g]
        if m.geom_type[g] == GeomType.MESH:
          gcom[g] = m.geom_pos[g] + R @ mc
          gI[g] = R @ mI @ R.T
        else:
          gcom[g] = m.geom_pos[g]
          gI[g] = R @ np.diag(m.geom_inertia_[g]) @ R.T
      com = sum(m.geom_mass_[g] * gcom[g] for g in geoms) / mass
      I = np.zeros((3, 3))
      for g in geoms:
        I += gI[g]
        dvec = gcom[g] - com
        I += m.geom_mass_[g] * (np.dot(dvec, dvec) * np.eye(3) - np.outer(dvec, dvec))
      m.body_mass[i] = mass
      m.body_ipos[i] = com
      if len(geoms) == 1 and m.geom_type[geoms[0]] != GeomType.MESH:
        # single geom: inertial frame = geom frame (diagonal inertia in geom frame)
        m.body_iquat[i] = m.geom_quat[geoms[0]]
        m.body_inertia[i] = m.geom_inertia_[geoms[0]]
      else:
        w, V = _eig3(I)
        m.body_iquat[i] = mat_to_quat(V)
        m.body_inertia[i] = w
    # <compiler boundmass / boundinertia>: lower bounds on every body except the world, flexcomp
    # vertex bodies included (MuJoCo user_body.cc; parity unpinned)
    if self.boundmass > 0:
      m.body_mass[1:] = np.maximum(m.body_mass[1:], self.boundmass)
    if self.boundinertia > 0:
      m.body_inertia[1:] = np.maximum(m.body_inertia[1:], self.boundinertia)

  def _subtreemass(self):
    m = self.m
    st = m.body_mass.copy()
    for i in range(m.nbody - 1, 0, -1):
      st[m.body_parentid[i]] += st[i]
    return st

  def _build_sites_cams_lights(self):
    m = self.m
    srows, crows, lrows = [], [], []
    for i, b in enumerate(self.bodies):
      for sa in b.sites:
        q = _orientation(sa, self.angle_scale, self.eulerseq)
        stype = {"sphere": GeomType.SPHERE, "capsule": GeomType.CAPSULE, "ellipsoid": GeomType.ELLIPSOID, "cylinder": GeomType.CYLINDER,
                 "box": GeomType.BOX}[sa.get("type", "sphere")]
        size = _merge_vec([0.005, 0.005, 0.005], _floats(sa.get("size", "0.005")))
        srows.append(dict(bodyid=i, pos=_floats(sa.get("pos", "0 0 0"), 3), quat=q if q is not None else [1, 0, 0, 0], name=sa.get("name", ""),
                          type=int(stype), size=size))
      for ca in b.cams:
        q = _orientation(ca, self.angle_scale, self.eulerseq)
        crows.append(
          dict(
            bodyid=i,
            name=ca.get("name", ""),
            mode=int(_CAMLIGHT_MODES[ca.get("mode", "fixed")]),
            target=ca.get("target"),
            pos=_floats(ca.get("pos", "0 0 0"), 3),
            quat=q if q is not None else [1, 0, 0, 0],
            fovy=float(ca.get("fovy", 45.0)),
            # camera intrinsics (mjsCamera: resolution 1 x 1, sensorsize 0 0, focal 0.01 m, principal 0; the
            # pixel forms convert through sensorsize / resolution): cam_resolution / cam_sensorsize /
            # cam_intrinsic, which the camprojection sensor reads (sensor.py:128-190)
            **_cam_intrinsics(ca),
          )
        )
      for la in b.lights:
        d = np.array(_floats(la.get("dir", "0 0 -1"), 3))
        d = d / max(np.linalg.norm(d), MJ_MINVAL)
        lrows.append(
          dict(
            bodyid=i,
            name=la.get("name", ""),
            mode=int(_CAMLIGHT_MODES[la.get("mode", "fixed")]),
            target=la.get("target"),
            pos=_floats(la.get("pos", "0 0 0"), 3),
            dir=d,
          )
        )
    name2body = {b.name: i for i, b in enumerate(self.bodies)}
    m.nsite = len(srows)
    m.site_names = [r["name"] for r in srows]
    m.site_bodyid = np.array([r["bodyid"] for r in srows], dtype=np.int32)
    m.site_pos = np.array([r["pos"] for r in srows]).reshape(-1, 3)
    m.site_quat = np.array([r["quat"] for r in srows]).reshape(-1, 4)
    m.site_type = np.array([r["type"] for r in srows], dtype=np.int32)  # the touch sensor's zone (sensor.py:2001-2076)
    m.site_size = np.array([r["size"] for r in srows], dtype=np.float64).reshape(-1, 3)
    m.ncam = len(crows)
    m.cam_names = [r["name"] for r in crows]
    m.cam_bodyid = np.array([r["bodyid"] for r in crows], dtype=np.int32)
    m.cam_mode = np.array([r["mode"] for r in crows], dtype=np.int32)
    m.cam_targetbodyid = np.array([name2body[r["target"]] if r["target"] else -1 for r in crows], dtype=np.int32)
    m.cam_pos = np.array([r["pos"] for r in crows]).reshape(-1, 3)
    m.cam_quat = np.array([r["quat"] for r in crows]).reshape(-1, 4)
    m.cam_fovy = np.array([r["fovy"] for r in crows])
    m.cam_resolution = np.array([r["resolution"] for r in crows], dtype=np.int32).reshape(-1, 2)
    m.cam_sensorsize = np.array([r["sensorsize"] for r in crows], dtype=np.float64).reshape(-1, 2)
    m.cam_intrinsic = np.array([r["intrinsic"] for r in crows], dtype=np.float64).reshape(-1, 4)
    m.nlight = len(lrows)
    m.light_names = [r["name"] for r in lrows]
    m.light_bodyid = np.array([r["bodyid"] for r in lrows], dtype=np.int32)
    m.light_mode = np.array([r["mode"] for r in lrows], dtype=np.int32)
    m.light_targetbodyid = np.array([name2body[r["target"]] if r["target"] else -1 for r in lrows], dtype=np.int32)
    m.light_pos = np.array([r["pos"] for r in lrows]).reshape(-1, 3)
    m.light_dir = np.array([r["dir"] for r in lrows]).reshape(-1, 3)

  def _build_tendons(self, root):
    """<tendon><fixed>: fixed (joint) tendons, length = sum coef * qpos (smooth.py:3085-3121); <tendon><spatial>:
    paths through sites, wrapping around sphere / cylinder geoms (optional sidesite) and split by pulleys
    (smooth.py:3172-3465).  The sparse Jacobian structure ten_J_rownnz / _rowadr / _colind lists each
    tendon's dofs ascending: the wrap joints' dofs (fixed), every dof on the kinematic chains of the path's
    bodies (spatial)."""
    m = self.m
    name2jnt = {n: i for i, n in enumerate(m.jnt_names) if n}
    name2site = {n: i for i, n in enumerate(m.site_names) if n}
    name2geom = {n: i for i, n in enumerate(m.geom_names) if n}
    rows, wraps = [], []
    for ten in root.findall("tendon"):
      for el in ten:
        if el.tag not in ("fixed", "spatial"):
          raise NotImplementedError(f"<tendon><{el.tag}> is not supported")
        a = dict(self.defaults[el.get("class", "main")].attrs.get("tendon", {}))
        a.update(el.attrib)

        def limited(key, rkey):
          v = a.get(key, "auto")
          if v == "auto":
            return bool(self.autolimits and rkey in a)
          return v == "true"

        adr = len(wraps)
        for j in el:
          if el.tag == "fixed":
            if j.tag != "joint":
              raise NotImplementedError(f"<fixed><{j.tag}> is not supported")
            jid = name2jnt[j.get("joint")]
            if m.jnt_type[jid] not in (JointType.HINGE, JointType.SLIDE):
              raise ValueError("fixed tendon joints must be hinge or slide joints")
            wraps.append((WrapType.JOINT, jid, float(j.get("coef", 1.0))))
          elif j.tag == "site":  # spatial tendon path (smooth.py:3172-3465): sites, wrap geoms, pulleys
            wraps.append((WrapType.SITE, name2site[j.get("site")], 0.0))
          elif j.tag == "geom":
            g = name2geom[j.get("geom")]
            gt = {GeomType.SPHERE: WrapType.SPHERE, GeomType.CYLINDER: WrapType.CYLINDER}.get(int(m.geom_type[g]))
            if gt is None:
              raise ValueError("spatial tendons wrap spheres and cylinders only")
            wraps.append((gt, g, float(name2site[j.get("sidesite")]) if j.get("sidesite") else -1.0))
          elif j.tag == "pulley":
            wraps.append((WrapType.PULLEY, -1, float(j.get("divisor", 1.0))))
          else:
            raise NotImplementedError(f"<spatial><{j.tag}> is not supported")
        if el.tag == "spatial":
          # every pulley-delimited branch runs site ... site, a wrap geom always between two sites
          kinds = [w[0] for w in wraps[adr:]]
          for i, k in enumerate(kinds):
            prv = kinds[i - 1] if i > 0 else WrapType.PULLEY
            nxt = kinds[i + 1] if i + 1 < len(kinds) else WrapType.PULLEY
            if k in (WrapType.SPHERE, WrapType.CYLINDER) and not (prv == WrapType.SITE and nxt == WrapType.SITE):
              raise ValueError("a spatial tendon's wrap geom sits between two sites")
            if k == WrapType.SITE and prv == WrapType.PULLEY and nxt == WrapType.PULLEY:
              raise ValueError("a spatial tendon branch needs two sites")
        sl = _floats(a.get("springlength", "-1 -1"))
        rows.append(dict(
          name=a.get("name", ""), adr=adr, num=len(wraps) - adr,
          stiffness=float(a.get("stiffness", 0.0)), damping=float(a.get("damping", 0.0)),
          frictionloss=float(a.get("frictionloss", 0.0)), armature=float(a.get("armature", 0.0)),
          limited=limited("limited", "range"), range=_floats(a.get("range", "0 0"), 2), margin=float(a.get("margin", 0.0)),
          springlength=sl if len(sl) == 2 else [sl[0], sl[0]],
          solref_lim=_merge_vec([0.02, 1.0], _floats(a.get("solreflimit", "0.02 1"))),
          solimp_lim=_merge_vec([0.9, 0.95, 0.001, 0.5, 2.0], _floats(a.get("solimplimit", "0.9 0.95 0.001 0.5 2"))),
          solref_fri=_merge_vec([0.02, 1.0], _floats(a.get("solreffriction", "0.02 1"))),
          solimp_fri=_merge_vec([0.9, 0.95, 0.001, 0.5, 2.0], _floats(a.get("solimpfriction", "0.9 0.95 0.001 0.5 2"))),
          actfrclimited=limited("actuatorfrclimited", "actuatorfrcrange"),
          actfrcrange=_floats(a.get("actuatorfrcrange", "0 0"), 2),
        ))
    nt = len(rows)
    m.ntendon, m.nwrap = nt, len(wraps)
    m.tendon_names = [r["name"] for r in rows]
    m.tendon_adr = np.array([r["adr"] for r in rows], dtype=np.int32)
    m.tendon_num = np.array([r["num"] for r in rows], dtype=np.int32)
    for k in ("stiffness", "damping", "frictionloss", "armature", "margin"):
      setattr(m, "tendon_" + k, np.array([r[k] for r in rows], dtype=np.float64))
    m.tendon_limited = np.array([r["limited"] for r in rows], dtype=bool)
    m.tendon_actfrclimited = np.array([r["actfrclimited"] for r in rows], dtype=bool)
    m.tendon_range = np.array([r["range"] for r in rows]).reshape(nt, 2)
    m.tendon_actfrcrange = np.array([r["actfrcrange"] for r in rows]).reshape(nt, 2)
    m.tendon_lengthspring = np.array([r["springlength"] for r in rows], dtype=np.float64).reshape(nt, 2)
    m.tendon_solref_lim = np.array([r["solref_lim"] for r in rows]).reshape(nt, 2)
    m.tendon_solimp_lim = np.array([r["solimp_lim"] for r in rows]).reshape(nt, 5)
    m.tendon_solref_fri = np.array([r["solref_fri"] for r in rows]).reshape(nt, 2)
    m.tendon_solimp_fri = np.array([r["solimp_fri"] for r in rows]).reshape(nt, 5)
    m.wrap_type = np.array([w[0] for w in wraps], dtype=np.int32)
    m.wrap_objid = np.array([w[1] for w in wraps], dtype=np.int32)
    m.wrap_prm = np.array([w[2] for w in wraps], dtype=np.float64)
    rownnz, rowadr, colind = [], [], []
    for r in rows:
      dofs = set()
      for k in range(r["adr"], r["adr"] + r["num"]):
        wt, obj = int(m.wrap_type[k]), int(m.wrap_objid[k])
        if wt == WrapType.JOINT:
          dofs.add(int(m.jnt_dofadr[obj]))
          continue
        # a spatial tendon moves with every dof on the chains of its sites' and wrap geoms' bodies
        b = -1 if wt == WrapType.PULLEY else int(m.site_bodyid[obj] if wt == WrapType.SITE else m.geom_bodyid[obj])
        while b > 0:
          dofs.update(range(int(m.body_dofadr[b]), int(m.body_dofadr[b]) + int(m.body_dofnum[b])))
          b = int(m.body_parentid[b])
      dofs = sorted(dofs)
      rowadr.append(len(colind))
      rownnz.append(len(dofs))
      colind += dofs
    m.ten_J_rownnz = np.array(rownnz, dtype=np.int32)
    m.ten_J_rowadr = np.array(rowadr, dtype=np.int32)
    m.ten_J_colind = np.array(colind, dtype=np.int32)
    m.nJten = len(colind)

  def _build_actuators(self, root):
    m = self.m
    name2jnt = {n: i for i, n in enumerate(m.jnt_names) if n}
    name2site = {n: i for i, n in enumerate(getattr(m, "site_names", [])) if n}
    rows = []
    for act in root.findall("actuator"):
      for el in act:
        if el.tag not in _ACTUATOR_TAGS:
          raise NotImplementedError(f"actuator <{el.tag}> not supported")
        cls = el.get("class", "main")
        a = dict(self.defaults[cls].attrs.get("actuator", {}))
        a.update(el.attrib)
        tag = el.tag
        gear = _merge_vec([1, 0, 0, 0, 0, 0], _floats(a.get("gear", "1")))
        ctrlrange = _floats(a.get("ctrlrange", "0 0"), 2)
        forcerange = _floats(a.get("forcerange", "0 0"), 2)
        actrange = _floats(a.get("actrange", "0 0"), 2)

        def limited(key, rkey):
          v = a.get(key, "auto")
          if v == "auto":
            return bool(self.autolimits and rkey in a)
          return v == "true"

        gainprm = np.zeros(10)
        biasprm = np.zeros(10)
        dynprm = np.zeros(10)
        dynprm[0] = 1.0
        gaintype, biastype, dyntype = GainType.FIXED, BiasType.NONE, DynType.NONE
        if tag == "motor":
          gainprm[0] = 1.0
        elif tag == "position":
          kp = float(a.get("kp", 1.0))
          kv = float(a.get("kv", 0.0))
          gainprm[0] = kp
          biastype = BiasType.AFFINE
          biasprm[:3] = [0.0, -kp, -kv]
          tc = float(a.get("timeconst", 0.0))
          if tc > 0:
            dyntype = DynType.FILTEREXACT
            dynprm[0] = tc
        elif tag == "velocity":
          kv = float(a.get("kv", 1.0))
          gainprm[0] = kv
          biastype = BiasType.AFFINE
          biasprm[:3] = [0.0, 0.0, -kv]
        elif tag == "damper":
          kv = float(a.get("kv", 1.0))
          gaintype = GainType.AFFINE
          gainprm[:3] = [0.0, 0.0, -kv]
        elif tag == "intvelocity":
          kp = float(a.get("kp", 1.0))
          gainprm[0] = kp
          biastype = BiasType.AFFINE
          biasprm[:3] = [0.0, -kp, 0.0]
          dyntype = DynType.INTEGRATOR
        elif tag == "adhesion":
          # MuJoCo's <adhesion> shortcut: gain * ctrl through a BODY transmission (smooth.py:2260-2273,
          # 2448-2602), ctrl limited to [0, ctrlrange[1]]
          gainprm[0] = float(a.get("gain", 1.0))
        elif tag == "muscle":
          # MuJoCo's <muscle> shortcut: muscle gain / bias / activation with its default curve
          # parameters, gainprm = biasprm = (range[2], force, scale, lmin, lmax, vmax, fpmax, fvmax) and
          # dynprm = (timeconst[2], tausmooth) (util_misc.py:478-600 unpacks them in this order)
          gaintype, biastype, dyntype = GainType.MUSCLE, BiasType.MUSCLE, DynType.MUSCLE
          tc = _floats(a.get("timeconst", "0.01 0.04"), 2)
          dynprm[:3] = [tc[0], tc[1], float(a.get("tausmooth", 0.0))]
          rng = _floats(a.get("range", "0.75 1.05"), 2)
          prm = [rng[0], rng[1], float(a.get("force", -1.0)), float(a.get("scale", 200.0)), float(a.get("lmin", 0.5)),
                 float(a.get("lmax", 1.6)), float(a.get("vmax", 1.5)), float(a.get("fpmax", 1.3)), float(a.get("fvmax", 1.2))]
          gainprm[:9] = prm
          biasprm[:9] = prm
        else:  # general
          gaintype = {"fixed": GainType.FIXED, "affine": GainType.AFFINE, "muscle": GainType.MUSCLE, "user": GainType.USER}[a.get("gaintype", "fixed")]
          biastype = {"none": BiasType.NONE, "affine": BiasType.AFFINE, "muscle": BiasType.MUSCLE, "user": BiasType.USER}[a.get("biastype", "none")]
          dyntype = {"none": DynType.NONE, "integrator": DynType.INTEGRATOR, "filter": DynType.FILTER, "filterexact": DynType.FILTEREXACT, "muscle": DynType.MUSCLE, "user": DynType.USER}[a.get("dyntype", "none")]
          gainprm[:] = _merge_vec([1] + [0] * 9, _floats(a.get("gainprm", "1")))
          biasprm[:] = _merge_vec([0] * 10, _floats(a.get("biasprm", "0")))
          dynprm[:] = _merge_vec([1] + [0] * 9, _floats(a.get("dynprm", "1")))
        if "joint" in a:
          trntype, trnid = TrnType.JOINT, [name2jnt[a["joint"]], -1]
        elif "jointinparent" in a:
          trntype, trnid = TrnType.JOINTINPARENT, [name2jnt[a["jointinparent"]], -1]
        elif "tendon" in a:
          trntype, trnid = TrnType.TENDON, [m.tendon_names.index(a["tendon"]), -1]
        elif "cranksite" in a:  # smooth.py:2150-2241
          trntype, trnid = TrnType.SLIDERCRANK, [name2site[a["cranksite"]], name2site[a["slidersite"]]]
        elif "site" in a:  # smooth.py:2274-2442
          trntype, trnid = TrnType.SITE, [name2site[a["site"]], name2site[a["refsite"]] if "refsite" in a else -1]
        elif "body" in a:  # smooth.py:2260-2273
          trntype, trnid = TrnType.BODY, [m.body_names.index(a["body"]), -1]
        else:
          raise ValueError(f"actuator <{tag}> names no transmission target")
        rows.append(
          dict(
            name=a.get("name", ""),
            trntype=int(trntype),
            trnid=trnid,
            gear=gear,
            gaintype=int(gaintype),
            biastype=int(biastype),
            dyntype=int(dyntype),
            gainprm=gainprm,
            biasprm=biasprm,
            dynprm=dynprm,
            ctrllimited=limited("ctrllimited", "ctrlrange"),
            forcelimited=limited("forcelimited", "forcerange"),
            actlimited=limited("actlimited", "actrange"),
            ctrlrange=ctrlrange,
            forcerange=forcerange,
            actrange=actrange,
            actearly=a.get("actearly", "false") == "true",
            lengthrange=_floats(a.get("lengthrange", "0 0"), 2),
            cranklength=float(a.get("cranklength", 0.0)),
          )
        )
    nu = len(rows)
    m.nu = nu
    m.actuator_names = [r["name"] for r in rows]
    m.actuator_trntype = np.array([r["trntype"] for r in rows], dtype=np.int32)
    m.actuator_trnid = np.array([r["trnid"] for r in rows], dtype=np.int32).reshape(nu, 2)
    m.actuator_gear = np.array([r["gear"] for r in rows]).reshape(nu, 6)
    m.actuator_gaintype = np.array([r["gaintype"] for r in rows], dtype=np.int32)
    m.actuator_biastype = np.array([r["biastype"] for r in rows], dtype=np.int32)
    m.actuator_dyntype = np.array([r["dyntype"] for r in rows], dtype=np.int32)
    m.actuator_gainprm = np.array([r["gainprm"] for r in rows]).reshape(nu, 10)
    m.actuator_biasprm = np.array([r["biasprm"] for r in rows]).reshape(nu, 10)
    m.actuator_dynprm = np.array([r["dynprm"] for r in rows]).reshape(nu, 10)
    m.actuator_ctrllimited = np.array([r["ctrllimited"] for r in rows], dtype=bool)
    m.actuator_forcelimited = np.array([r["forcelimited"] for r in rows], dtype=bool)
    m.actuator_actlimited = np.array([r["actlimited"] for r in rows], dtype=bool)
    m.actuator_ctrlrange = np.array([r["ctrlrange"] for r in rows]).reshape(nu, 2)
    m.actuator_forcerange = np.array([r["forcerange"] for r in rows]).reshape(nu, 2)
    m.actuator_actrange = np.array([r["actrange"] for r in rows]).reshape(nu, 2)
    m.actuator_actearly = np.array([r["actearly"] for r in rows], dtype=bool)
    m.actuator_cranklength = np.array([r["cranklength"] for r in rows], dtype=np.float64)
    m.actuator_lengthrange = np.array([r["lengthrange"] for r in rows], dtype=np.float64).reshape(nu, 2)
    # muscles need the actuator length range (mj_setLengthRange).  MuJoCo finds it at compile time by
    # simulation; here it is the transmission's limited range times the gear (MuJoCo's `uselimit`
    # path), unless the element gives lengthrange itself
    for i, r in enumerate(rows):
      is_muscle = r["dyntype"] == DynType.MUSCLE or r["gaintype"] == GainType.MUSCLE or r["biastype"] == BiasType.MUSCLE
      if not is_muscle or m.actuator_lengthrange[i, 0] < m.actuator_lengthrange[i, 1]:
        continue
      g = r["gear"][0]
      rng = None
      if r["trntype"] in (TrnType.JOINT, TrnType.JOINTINPARENT) and m.jnt_limited[r["trnid"][0]]:
        rng = m.jnt_range[r["trnid"][0]]
      elif r["trntype"] == TrnType.TENDON and m.tendon_limited[r["trnid"][0]]:
        rng = m.tendon_range[r["trnid"][0]]
      if rng is not None:
        m.actuator_lengthrange[i] = sorted((g * rng[0], g * rng[1]))
    actadr = -np.ones(nu, dtype=np.int32)
    actnum = np.zeros(nu, dtype=np.int32)
    na = 0
    for i, r in enumerate(rows):
      if r["dyntype"] != DynType.NONE:
        actadr[i] = na
        actnum[i] = 1
        na += 1
    m.actuator_actadr, m.actuator_actnum, m.na = actadr, actnum, na

  def _build_equality(self, root):
    """<equality>: connect (constraint.py:124-365), weld (:792-1110) and joint (:367-495) couplings.

    eq_data follows MuJoCo's layout: connect = (anchor1, anchor2); weld = (anchor, relpose pos,
    relpose quat, torquescale).  The offsets MuJoCo derives at qpos0 (connect anchor2, weld relpose
    when its quaternion is zero) are filled in by set_const."""
    m = self.m
    name2jnt = {n: i for i, n in enumerate(m.jnt_names)}
    name2body = {n: i for i, n in enumerate(m.body_names)}
    name2site = {n: i for i, n in enumerate(getattr(m, "site_names", []))}
    rows = []
    # <flexcomp><edge equality="true"/>: one FLEX equality per flex, added when the flexcomp is
    # parsed, i.e. ahead of the <equality> section (constraint.py:677-790 reads eq_obj1id = flex id)
    for f, fc in enumerate(self.flexcomps):
      if fc["edge_equality"]:
        rows.append(dict(name="", type=int(EqType.FLEX), obj1=f, obj2=-1, objtype=int(ObjType.UNKNOWN), data=np.zeros(11),
                         solref=fc["edge_solref"], solimp=fc["edge_solimp"], active=True))
    for eq in root.findall("equality"):
      for el in eq:
        a = dict(self.defaults[el.get("class", "main")].attrs.get("equality", {}))
        a.update(el.attrib)
        data = np.zeros(11)
        objtype = int(ObjType.JOINT)
        if el.tag == "joint":
          etype, obj1 = EqType.JOINT, name2jnt[a["joint1"]]
          obj2 = name2jnt[a["joint2"]] if "joint2" in a else -1
          data[:5] = _merge_vec([0, 1, 0, 0, 0], _floats(a.get("polycoef", "0 1 0 0 0")))
        elif el.tag == "tendon":  # constraint.py:498-674: length1 - length0_1 = poly(length2 - length0_2)
          etype, objtype = EqType.TENDON, int(ObjType.TENDON)
          obj1 = m.tendon_names.index(a["tendon1"])
          obj2 = m.tendon_names.index(a["tendon2"]) if "tendon2" in a else -1
          data[:5] = _merge_vec([0, 1, 0, 0, 0], _floats(a.get("polycoef", "0 1 0 0 0")))
        elif el.tag in ("connect", "weld"):
          etype = EqType.CONNECT if el.tag == "connect" else EqType.WELD
          if "site1" in a:
            objtype, obj1 = int(ObjType.SITE), name2site[a["site1"]]
            obj2 = name2site[a["site2"]]
          else:
            objtype, obj1 = int(ObjType.BODY), name2body[a["body1"]]
            obj2 = name2body[a["body2"]] if "body2" in a else 0
          data[:3] = _floats(a.get("anchor", "0 0 0"), 3)
          if etype == EqType.WELD:
            data[3:10] = _merge_vec([0, 1, 0, 0, 0, 0, 0], _floats(a.get("relpose", "0 1 0 0 0 0 0")))
            data[10] = float(a.get("torquescale", 1.0))
        else:
          raise NotImplementedError(f"<equality><{el.tag}> is not supported by the MJCF compiler yet")
        rows.append(dict(
          name=a.get("name", ""), type=int(etype), obj1=obj1, obj2=obj2, objtype=objtype, data=data,
          solref=_merge_vec([0.02, 1.0], _floats(a.get("solref", "0.02 1"))),
          solimp=_merge_vec([0.9, 0.95, 0.001, 0.5, 2.0], _floats(a.get("solimp", "0.9 0.95 0.001 0.5 2"))),
          active=a.get("active", "true") == "true"))
    m.neq = len(rows)
    m.eq_names = [r["name"] for r in rows]
    m.eq_type = np.array([r["type"] for r in rows], dtype=np.int32)
    m.eq_obj1id = np.array([r["obj1"] for r in rows], dtype=np.int32)
    m.eq_obj2id = np.array([r["obj2"] for r in rows], dtype=np.int32)
    m.eq_objtype = np.array([r["objtype"] for r in rows], dtype=np.int32)
    m.eq_data = np.array([r["data"] for r in rows]).reshape(m.neq, 11)
    m.eq_solref = np.array([r["solref"] for r in rows]).reshape(m.neq, 2)
    m.eq_solimp = np.array([r["solimp"] for r in rows]).reshape(m.neq, 5)
    m.eq_active0 = np.array([r["active"] for r in rows], dtype=np.uint8)

  # <sensor> element -> (type, dim, datatype, needstage, object attribute, objtype)
  _SENSORS = {
    "accelerometer": (SensorType.ACCELEROMETER, 3, DataType.REAL, Stage.ACC, "site", ObjType.SITE),
    "velocimeter": (SensorType.VELOCIMETER, 3, DataType.REAL, Stage.VEL, "site", ObjType.SITE),
    "gyro": (SensorType.GYRO, 3, DataType.REAL, Stage.VEL, "site", ObjType.SITE),
    "force": (SensorType.FORCE, 3, DataType.REAL, Stage.ACC, "site", ObjType.SITE),
    "torque": (SensorType.TORQUE, 3, DataType.REAL, Stage.ACC, "site", ObjType.SITE),
    "magnetometer": (SensorType.MAGNETOMETER, 3, DataType.REAL, Stage.POS, "site", ObjType.SITE),
    "jointpos": (SensorType.JOINTPOS, 1, DataType.REAL, Stage.POS, "joint", ObjType.JOINT),
    "jointvel": (SensorType.JOINTVEL, 1, DataType.REAL, Stage.VEL, "joint", ObjType.JOINT),
    "actuatorpos": (SensorType.ACTUATORPOS, 1, DataType.REAL, Stage.POS, "actuator", ObjType.ACTUATOR),
    "actuatorvel": (SensorType.ACTUATORVEL, 1, DataType.REAL, Stage.VEL, "actuator", ObjType.ACTUATOR),
    "actuatorfrc": (SensorType.ACTUATORFRC, 1, DataType.REAL, Stage.ACC, "actuator", ObjType.ACTUATOR),
    "jointactuatorfrc": (SensorType.JOINTACTFRC, 1, DataType.REAL, Stage.ACC, "joint", ObjType.JOINT),
    "ballquat": (SensorType.BALLQUAT, 4, DataType.QUATERNION, Stage.POS, "joint", ObjType.JOINT),
    "ballangvel": (SensorType.BALLANGVEL, 3, DataType.REAL, Stage.VEL, "joint", ObjType.JOINT),
    "framepos": (SensorType.FRAMEPOS, 3, DataType.REAL, Stage.POS, None, None),
    "framequat": (SensorType.FRAMEQUAT, 4, DataType.QUATERNION, Stage.POS, None, None),
    "framexaxis": (SensorType.FRAMEXAXIS, 3, DataType.AXIS, Stage.POS, None, None),
    "frameyaxis": (SensorType.FRAMEYAXIS, 3, DataType.AXIS, Stage.POS, None, None),
    "framezaxis": (SensorType.FRAMEZAXIS, 3, DataType.AXIS, Stage.POS, None, None),
    "framelinvel": (SensorType.FRAMELINVEL, 3, DataType.REAL, Stage.VEL, None, None),
    "frameangvel": (SensorType.FRAMEANGVEL, 3, DataType.REAL, Stage.VEL, None, None),
    "framelinacc": (SensorType.FRAMELINACC, 3, DataType.REAL, Stage.ACC, None, None),
    "frameangacc": (SensorType.FRAMEANGACC, 3, DataType.REAL, Stage.ACC, None, None),
    "subtreecom": (SensorType.SUBTREECOM, 3, DataType.REAL, Stage.POS, "body", ObjType.BODY),
    "clock": (SensorType.CLOCK, 1, DataType.REAL, Stage.POS, None, ObjType.UNKNOWN),
    "touch": (SensorType.TOUCH, 1, DataType.POSITIVE, Stage.ACC, "site", ObjType.SITE),
    "tendonpos": (SensorType.TENDONPOS, 1, DataType.REAL, Stage.POS, "tendon", ObjType.TENDON),
    "tendonvel": (SensorType.TENDONVEL, 1, DataType.REAL, Stage.VEL, "tendon", ObjType.TENDON),
    "tendonactuatorfrc": (SensorType.TENDONACTFRC, 1, DataType.REAL, Stage.ACC, "tendon", ObjType.TENDON),
    "jointlimitpos": (SensorType.JOINTLIMITPOS, 1, DataType.REAL, Stage.POS, "joint", ObjType.JOINT),
    "jointlimitvel": (SensorType.JOINTLIMITVEL, 1, DataType.REAL, Stage.VEL, "joint", ObjType.JOINT),
    "jointlimitfrc": (SensorType.JOINTLIMITFRC, 1, DataType.POSITIVE, Stage.ACC, "joint", ObjType.JOINT),
    "tendonlimitpos": (SensorType.TENDONLIMITPOS, 1, DataType.REAL, Stage.POS, "tendon", ObjType.TENDON),
    "tendonlimitvel": (SensorType.TENDONLIMITVEL, 1, DataType.REAL, Stage.VEL, "tendon", ObjType.TENDON),
    "tendonlimitfrc": (SensorType.TENDONLIMITFRC, 1, DataType.POSITIVE, Stage.ACC, "tendon", ObjType.TENDON),
    "subtreelinvel": (SensorType.SUBTREELINVEL, 3, DataType.REAL, Stage.VEL, "body", ObjType.BODY),
    "subtreeangmom": (SensorType.SUBTREEANGMOM, 3, DataType.REAL, Stage.VEL, "body", ObjType.BODY),
    "e_potential": (SensorType.E_POTENTIAL, 1, DataType.REAL, Stage.POS, None, ObjType.UNKNOWN),
    "e_kinetic": (SensorType.E_KINETIC, 1, DataType.REAL, Stage.VEL, None, ObjType.UNKNOWN),
    # collision sensors: geom1 | body1 against geom2 | body2 (MuJoCo's mjSENS_GEOMDIST / GEOMNORMAL / GEOMFROMTO)
    "distance": (SensorType.GEOMDIST, 1, DataType.REAL, Stage.POS, "collision", None),
    "normal": (SensorType.GEOMNORMAL, 3, DataType.AXIS, Stage.POS, "collision", None),
    "fromto": (SensorType.GEOMFROMTO, 6, DataType.REAL, Stage.POS, "collision", None),
    # insidesite: objtype / objname inside the geometry of `site`
    "insidesite": (SensorType.INSIDESITE, 1, DataType.REAL, Stage.POS, "insidesite", None),
    # contact: matched contacts' data (sensor.py:1750-1940, 2275-2430); dim from num x the data fields
    "contact": (SensorType.CONTACT, 0, DataType.REAL, Stage.ACC, "contact", None),
    # camprojection: pixel coordinates of `site` in `camera`'s image (sensor.py:128-190)
    "camprojection": (SensorType.CAMPROJECTION, 2, DataType.REAL, Stage.POS, "camprojection", ObjType.SITE),
    # tactile: per vertex of `mesh` placed on `geom`, the penetration pressure and tangential slip of the
    # geoms in contact with that geom's weld body (sensor.py:2085-2250); dim = 3 x vertices
    "tactile": (SensorType.TACTILE, 0, DataType.REAL, Stage.ACC, "tactile", ObjType.MESH),
  }
  _OBJTYPES = {"body": ObjType.BODY, "xbody": ObjType.XBODY, "geom": ObjType.GEOM, "site": ObjType.SITE, "camera": ObjType.CAMERA}

  def _build_sensors(self, root):
    """<sensor>: the sensor table (mjModel sensor_* fields; sensor.py reads them)."""
    m = self.m
    names = {
      ObjType.BODY: {n: i for i, n in enumerate(m.body_names)},
      ObjType.XBODY: {n: i for i, n in enumerate(m.body_names)},
      ObjType.GEOM: {n: i for i, n in enumerate(m.geom_names) if n},
      ObjType.SITE: {n: i for i, n in enumerate(m.site_names) if n},
      ObjType.CAMERA: {n: i for i, n in enumerate(m.cam_names) if n},
      ObjType.JOINT: {n: i for i, n in enumerate(m.jnt_names) if n},
      ObjType.ACTUATOR: {n: i for i, n in enumerate(m.actuator_names) if n},
      ObjType.TENDON: {n: i for i, n in enumerate(getattr(m, "tendon_names", [])) if n},
    }
    rows = []
    adr = 0
    for sec in root.findall("sensor"):
      for el in sec:
        if el.tag not in self._SENSORS:
          raise NotImplementedError(f"sensor <{el.tag}> is not supported by this build yet")
        a = dict(self.defaults[el.get("class", "main")].attrs.get("sensor", {}))
        a.update(el.attrib)
        stype, dim, dtype, stage, key, otype = self._SENSORS[el.tag]
        objid, reftype, refid = -1, ObjType.UNKNOWN, -1
        intprm = [0, 0, 0]
        if key == "collision":
          otype, objid = (ObjType.GEOM, names[ObjType.GEOM][a["geom1"]]) if "geom1" in a else (ObjType.BODY, names[ObjType.BODY][a["body1"]])
          reftype, refid = (ObjType.GEOM, names[ObjType.GEOM][a["geom2"]]) if "geom2" in a else (ObjType.BODY, names[ObjType.BODY][a["body2"]])
        elif key == "contact":
          # obj: geom1 | body1 | subtree1 | site, ref: geom2 | body2 | subtree2 (either may be absent: UNKNOWN);
          # intprm = (data field bits: found force torque dist pos normal tangent, reduce: none mindist
          # maxforce netforce, 0) -- MuJoCo's mjtConDataField / mjtConReduce
          otype, objid = ObjType.UNKNOWN, -1
          for k_, t_ in (("geom1", ObjType.GEOM), ("body1", ObjType.BODY), ("subtree1", ObjType.XBODY), ("site", ObjType.SITE)):
            if k_ in a:
              otype, objid = t_, names[ObjType.BODY if t_ == ObjType.XBODY else t_][a[k_]]
          for k_, t_ in (("geom2", ObjType.GEOM), ("body2", ObjType.BODY), ("subtree2", ObjType.XBODY)):
            if k_ in a:
              reftype, refid = t_, names[ObjType.BODY if t_ == ObjType.XBODY else t_][a[k_]]
          fields = a.get("data", "found").split()
          order = ["found", "force", "torque", "dist", "pos", "normal", "tangent"]
          if any(f_ not in order for f_ in fields) or [order.index(f_) for f_ in fields] != sorted(order.index(f_) for f_ in fields):
            raise ValueError(f"contact sensor data {fields}: fields must be among {order}, in that order")
          spec = sum(1 << order.index(f_) for f_ in fields)
          size = sum((1, 3, 3, 1, 3, 3, 3)[order.index(f_)] for f_ in fields)
          reduce = ["none", "mindist", "maxforce", "netforce"].index(a.get("reduce", "none"))
          num = int(a.get("num", 1))
          if reduce == 3 and num != 1:
            raise ValueError("contact sensor: reduce='netforce' takes num = 1")
          dim = num * size
          intprm = [spec, reduce, 0]
        elif key == "camprojection":
          objid = names[ObjType.SITE][a["site"]]
          reftype, refid = ObjType.CAMERA, names[ObjType.CAMERA][a["camera"]]
        elif key == "tactile":
          objid = self.mesh_id[a["mesh"]]
          reftype, refid = ObjType.GEOM, names[ObjType.GEOM][a["geom"]]
          dim = 3 * int(m.mesh_vertnum[objid])
        elif key == "insidesite":
          otype = self._OBJTYPES[a["objtype"]]
          objid = names[otype][a["objname"]]
          reftype, refid = ObjType.SITE, names[ObjType.SITE][a["site"]]
        elif key is not None:
          objid = names[otype][a[key]]
        elif otype is None:  # frame sensors: objtype / objname (+ optional reftype / refname)
          otype = self._OBJTYPES[a["objtype"]]
          objid = names[otype][a["objname"]]
          if "refname" in a:
            reftype = self._OBJTYPES[a["reftype"]]
            refid = names[reftype][a["refname"]]
        rows.append(dict(name=a.get("name", ""), type=int(stype), datatype=int(dtype), needstage=int(stage), objtype=int(otype),
                         objid=objid, reftype=int(reftype), refid=refid, dim=dim, adr=adr, cutoff=float(a.get("cutoff", 0.0)),
                         noise=float(a.get("noise", 0.0)), intprm=intprm))
        adr += dim
    m.nsensor = len(rows)
    m.nsensordata = adr
    m.sensor_names = [r["name"] for r in rows]
    for f in ("type", "datatype", "needstage", "objtype", "objid", "reftype", "refid", "dim", "adr"):
      setattr(m, "sensor_" + f, np.array([r[f] for r in rows], dtype=np.int32))
    m.sensor_intprm = np.array([r["intprm"] for r in rows], dtype=np.int32).reshape(-1, 3)
    m.sensor_cutoff = np.array([r["cutoff"] for r in rows], dtype=np.float64)
    m.sensor_noise = np.array([r["noise"] for r in rows], dtype=np.float64)

  def _build_contact(self, root):
    m = self.m
    name2body = {b.name: i for i, b in enumerate(self.bodies)}
    name2geom = {n: i for i, n in enumerate(m.geom_names) if n}
    sigs, pairs = [], []
    for c in root.findall("contact"):
      for el in c:
        if el.tag == "exclude":
          b1, b2 = name2body[el.get("body1")], name2body[el.get("body2")]
          b1, b2 = min(b1, b2), max(b1, b2)
          sigs.append((b1 << 16) + b2)
        elif el.tag == "pair":
          pairs.append(self._pair(self._resolve("pair", el, None), name2geom))
    m.exclude_signature = np.array(sigs, dtype=np.int32)
    m.nexclude = len(sigs)
    m.npair = len(pairs)
    m.pair_geom1 = np.array([p["geom1"] for p in pairs], dtype=np.int32)
    m.pair_geom2 = np.array([p["geom2"] for p in pairs], dtype=np.int32)
    m.pair_dim = np.array([p["dim"] for p in pairs], dtype=np.int32)
    for f, n in (("friction", 5), ("solref", 2), ("solreffriction", 2), ("solimp", 5)):
      setattr(m, "pair_" + f, np.array([p[f] for p in pairs], dtype=np.float64).reshape(len(pairs), n))
    m.pair_margin = np.array([p["margin"] for p in pairs], dtype=np.float64)
    m.pair_gap = np.array([p["gap"] for p in pairs], dtype=np.float64)

  def _pair(self, a, name2geom):
    """One explicit <contact><pair>: attributes it leaves unset are derived from its two geoms the way
    MuJoCo's compiler does (mjCPair::Compile): margin / gap = max, condim / friction / solref / solimp
    from the higher-priority geom, or at equal priority max condim and friction and solmix-weighted
    solref / solimp (min solref when either is a direct (negative) reference); solreffriction = 0 0.
    The compiled values feed contact_params' pair branch (collision_core.py:270-277)."""
    m = self.m
    g1, g2 = name2geom[a["geom1"]], name2geom[a["geom2"]]
    out = dict(geom1=g1, geom2=g2)
    out["margin"] = float(a["margin"]) if "margin" in a else max(m.geom_margin[g1], m.geom_margin[g2])
    out["gap"] = float(a["gap"]) if "gap" in a else max(m.geom_gap[g1], m.geom_gap[g2])
    p1, p2 = m.geom_priority[g1], m.geom_priority[g2]
    if p1 != p2:
      gh = g1 if p1 > p2 else g2
      dim = m.geom_condim[gh]
      fr = m.geom_friction[gh]
      sref, simp = m.geom_solref[gh], m.geom_solimp[gh]
    else:
      dim = max(m.geom_condim[g1], m.geom_condim[g2])
      fr = np.maximum(m.geom_friction[g1], m.geom_friction[g2])
      s1, s2 = m.geom_solmix[g1], m.geom_solmix[g2]
      if s1 >= MJ_MINVAL and s2 >= MJ_MINVAL:
        mix = s1 / (s1 + s2)
      elif s1 < MJ_MINVAL and s2 < MJ_MINVAL:
        mix = 0.5
      else:
        mix = 0.0 if s1 < MJ_MINVAL else 1.0
      r1, r2 = m.geom_solref[g1], m.geom_solref[g2]
      sref = mix * r1 + (1 - mix) * r2 if (r1[0] > 0 and r2[0] > 0) else np.minimum(r1, r2)
      simp = mix * m.geom_solimp[g1] + (1 - mix) * m.geom_solimp[g2]
    out["dim"] = int(a["condim"]) if "condim" in a else int(dim)
    out["friction"] = _merge_vec([fr[0], fr[0], fr[1], fr[2], fr[2]], _floats(a["friction"])) if "friction" in a else \
      [fr[0], fr[0], fr[1], fr[2], fr[2]]
    out["solref"] = _merge_vec([0.02, 1.0], _floats(a["solref"])) if "solref" in a else list(sref)
    out["solimp"] = _merge_vec([0.9, 0.95, 0.001, 0.5, 2.0], _floats(a["solimp"])) if "solimp" in a else list(simp)
    out["solreffriction"] = _merge_vec([0.0, 0.0], _floats(a["solreffriction"])) if "solreffriction" in a else [0.0, 0.0]
    return out

  def _build_keys(self, root):
    m = self.m
    keys = []
    for kf in root.findall("keyframe"):
      for k in kf.findall("key"):
        keys.append(k)
    m.nkey = len(keys)
    m.key_names = [k.get("name", "") for k in keys]
    m.key_time = np.array([float(k.get("time", 0.0)) for k in keys])
    # a key shorter than nq (flexcomp dofs are appended after the keyed joints) is completed with qpos0
    m.key_qpos = np.array([np.concatenate([_floats(k.get("qpos")), m.qpos0[len(_floats(k.get("qpos"))):]]) if k.get("qpos") else m.qpos0
                           for k in keys]).reshape(m.nkey, m.nq)
    # a (near-)zero free / ball joint quaternion in a key is the identity, as MuJoCo's mju_normalize4 makes
    # it (the reference's aloha_pot keys store 0 0 0 0 for the pot's free joint, which the MuJoCo-C fixture
    # state of unroll_test.py:42 reads as the identity); other key quaternions are kept as written
    for j in range(m.njnt):
      if int(m.jnt_type[j]) in (0, 1):  # FREE, BALL
        a = int(m.jnt_qposadr[j]) + (3 if int(m.jnt_type[j]) == 0 else 0)
        for kq in m.key_qpos:
          if float(np.linalg.norm(kq[a:a + 4])) < MJ_MINVAL:
            kq[a:a + 4] = (1.0, 0.0, 0.0, 0.0)
    m.key_qvel = np.array([_floats(k.get("qvel")) if k.get("qvel") else np.zeros(m.nv) for k in keys]).reshape(m.nkey, m.nv)
    m.key_act = np.array([_floats(k.get("act")) if k.get("act") else np.zeros(m.na) for k in keys]).reshape(m.nkey, m.na)
    m.key_ctrl = np.array([_floats(k.get("ctrl")) if k.get("ctrl") else np.zeros(m.nu) for k in keys]).reshape(m.nkey, m.nu)
    m.key_mpos = np.zeros((m.nkey, 3 * m.nmocap))
    m.key_mquat = np.tile(np.tile([1.0, 0, 0, 0], m.nmocap), (m.nkey, 1))


def _cam_intrinsics(ca):
  """resolution / sensorsize / intrinsic = [focal x, focal y, principal x, principal y] (length units) of a
  <camera>: focal / principal in length, or focalpixel / principalpixel converted by sensorsize / resolution."""
  res = [int(round(x)) for x in _floats(ca.get("resolution", "1 1"), 2)]
  ss = _floats(ca.get("sensorsize", "0 0"), 2)
  focal = _floats(ca.get("focal", "0.01 0.01"), 2)
  principal = _floats(ca.get("principal", "0 0"), 2)
  if "focalpixel" in ca:
    fp = _floats(ca["focalpixel"], 2)
    focal = [fp[i] / max(res[i], 1) * ss[i] for i in range(2)]
  if "principalpixel" in ca:
    pp = _floats(ca["principalpixel"], 2)
    principal = [pp[i] / max(res[i], 1) * ss[i] for i in range(2)]
  return dict(resolution=res, sensorsize=ss, intrinsic=list(focal) + list(principal))


def _read_png(path):
  """(height, width, samples (h, w, channels), bit depth) of a PNG file: the chunk stream, zlib and the five
  scanline filters (PNG spec 9.2), for 8 / 16-bit greyscale, grey + alpha, RGB and RGBA images."""
  import struct
  import zlib

  with open(path, "rb") as f:
    raw = f.read()
  if raw[:8] != b"\x89PNG\r\n\x1a\n":
    raise ValueError(f"{path}: not a PNG file")
  pos, idat, hdr = 8, [], None
  while pos < len(raw):
    n = struct.unpack(">I", raw[pos:pos + 4])[0]
    kind, body = raw[pos + 4:pos + 8], raw[pos + 8:pos + 8 + n]
    pos += 12 + n
    if kind == b"IHDR":
      hdr = struct.unpack(">IIBBBBB", body)
    elif kind == b"IDAT":
      idat.append(body)
    elif kind == b"IEND":
      break
  w, h, depth, ctype, _, _, interlace = hdr
  chans = {0: 1, 2: 3, 4: 2, 6: 4}.get(ctype)
  if chans is None or depth not in (8, 16) or interlace:
    raise NotImplementedError(f"{path}: PNG color type {ctype}, bit depth {depth}, interlace {interlace} not supported")
  bpp = chans * depth // 8
  stride = w * bpp
  data = zlib.decompress(b"".join(idat))
  out = np.zeros((h, stride), dtype=np.int32)
  prev = np.zeros(stride, dtype=np.int32)
  for r in range(h):
    ft = data[r * (stride + 1)]
    line = np.frombuffer(data, dtype=np.uint8, count=stride, offset=r * (stride + 1) + 1).astype(np.int32)
    cur = np.zeros(stride, dtype=np.int32)
    if ft == 0:
      cur = line
    elif ft == 2:
      cur = (line + prev) & 255
    else:
      for i in range(stride):  # sub / average / paeth depend on the reconstructed left byte
        left = cur[i - bpp] if i >= bpp else 0
        up, ul = prev[i], (prev[i - bpp] if i >= bpp else 0)
        if ft == 1:
          pr = left
        elif ft == 3:
          pr = (left + up) >> 1
        else:
          p = left + up - ul
          pa, pb, pc = abs(p - left), abs(p - up), abs(p - ul)
          pr = left if (pa <= pb and pa <= pc) else (up if pb <= pc else ul)
        cur[i] = (line[i] + pr) & 255
    out[r] = cur
    prev = cur
  px = out.reshape(h, w, bpp).astype(np.uint16)
  if depth == 16:
    px = (px[:, :, 0::2] << 8) | px[:, :, 1::2]
  return h, w, px.reshape(h, w, chans), depth


def _read_hfield_file(path):
  """(nrow, ncol, elevation) of an <hfield file=...>, in hfield_data order (row 0 at -y).  PNG: decoded to
  8-bit grey as MuJoCo's loader does (lodepng LCT_GREY: the red / grey channel, 16-bit samples by their
  high byte), image row 0 -- the top -- becoming the last grid row, values / 255.  Any other extension:
  MuJoCo's binary format, int32 nrow, int32 ncol, then nrow * ncol float32 values in grid order."""
  if path.lower().endswith(".png"):
    h, w, px, depth = _read_png(path)
    grey = (px[:, :, 0] >> 8) if depth == 16 else px[:, :, 0]
    return h, w, (grey[::-1].astype(np.float64) / 255.0).reshape(-1)
  with open(path, "rb") as f:
    raw = f.read()
  nrow, ncol = np.frombuffer(raw[:8], dtype="<i4")
  data = np.frombuffer(raw[8:8 + 4 * int(nrow) * int(ncol)], dtype="<f4").astype(np.float64)
  return int(nrow), int(ncol), data


# the local edge order of one element (passive.py:606-613)
_FLEX_LOCAL_EDGES = {1: ((0, 1),), 2: ((1, 2), (2, 0), (0, 1)), 3: ((0, 1), (1, 2), (2, 0), (2, 3), (0, 3), (1, 3))}


def _body_world_pos(b):
  """World position of a compiler body at qpos0 (its frame chain up to the world body)."""
  p = np.zeros(3)
  while b is not None and b.parent is not None:
    p = quat_to_mat(np.asarray(b.quat, dtype=float)) @ p + np.asarray(b.pos, dtype=float)
    b = b.parent
  return p


def _svk_metric(X, young, poisson, dim, thickness, radius):
  """Edge metric M (nedge x nedge) of one flex element with rest vertices X ((dim+1) x 3) such that
  its Saint Venant-Kirchhoff energy is 1/4 s' M s, s_e = L_e^2 - L0_e^2 over the local edges.

  With g_i the barycentric gradients of the rest element (sum_i g_i = 0), the right Cauchy-Green
  tensor is C = F'F = -sum_{i<j} L_ij^2 S_ij, S_ij = (g_i g_j' + g_j g_i') / 2, so the Green strain is
  E = -1/2 sum_e s_e S_e and W = V (mu tr E^2 + lambda/2 (tr E)^2) gives
  M[e1, e2] = V (mu tr(S_e1 S_e2) + lambda/2 tr(S_e1) tr(S_e2)).  dim 3: V the tetrahedron volume;
  dim 2: V = area * thickness with the plane-stress lambda 2 lambda mu / (lambda + 2 mu) (the gradients
  in the triangle's plane); dim 1: V = length * pi radius^2 and the axial modulus (M = young V tr(S)^2 / 2)."""
  X = np.asarray(X, dtype=float)
  D = (X[1:] - X[0]).T  # 3 x dim
  G = np.linalg.pinv(D)  # dim x 3: rows = gradients of the barycentric coordinates 1..dim
  g = np.vstack([-G.sum(axis=0), G])
  lam = young * poisson / ((1.0 + poisson) * (1.0 - 2.0 * poisson)) if poisson < 0.5 else 0.0
  mu = young / (2.0 * (1.0 + poisson))
  if dim == 3:
    vol = abs(np.linalg.det(D)) / 6.0
  elif dim == 2:
    vol = 0.5 * np.linalg.norm(np.cross(D[:, 0], D[:, 1])) * thickness
    lam = 2.0 * lam * mu / (lam + 2.0 * mu)
  else:
    vol = np.linalg.norm(D[:, 0]) * np.pi * radius * radius
  S = [0.5 * (np.outer(g[i], g[j]) + np.outer(g[j], g[i])) for i, j in _FLEX_LOCAL_EDGES[dim]]
  n = len(S)
  M = np.zeros((n, n))
  for a in range(n):
    for b in range(n):
      if dim == 1:
        M[a, b] = 0.5 * young * vol * np.trace(S[a]) * np.trace(S[b])
      else:
        M[a, b] = vol * (mu * np.trace(S[a] @ S[b]) + 0.5 * lam * np.trace(S[a]) * np.trace(S[b]))
  return M


def _vertex_normals(v, f):
  """Unit vertex normals: the sum of the adjacent triangles' (area-weighted) normals."""
  n = np.zeros((len(v), 3))
  f = np.asarray(f, dtype=np.int64).reshape(-1, 3)
  if len(f):
    fn = np.cross(v[f[:, 1]] - v[f[:, 0]], v[f[:, 2]] - v[f[:, 0]])
    for k in range(3):
      np.add.at(n, f[:, k], fn)
  ln = np.linalg.norm(n, axis=1, keepdims=True)
  return np.where(ln > 0, n / np.maximum(ln, 1e-30), np.array([0.0, 0.0, 1.0]))


def _bending_coef(x, mu, thickness):
  """16 coefficients of the quadratic bending energy of one interior edge: x = (edge v0, edge v1,
  flap of triangle 0, flap of triangle 1).  Q = c c' * mu h^3 / (8 (A0 + A1)), c the cotangent
  weights; Q annihilates translations and any flat configuration of the four vertices."""
  e0, e1, e2, e3, e4 = x[1] - x[0], x[2] - x[0], x[3] - x[0], x[2] - x[1], x[3] - x[1]

  def cot(a, b):
    return float(np.dot(a, b) / max(np.linalg.norm(np.cross(a, b)), MJ_MINVAL))

  c01, c02, c03, c04 = cot(e0, e1), cot(e0, e2), cot(-e0, e3), cot(-e0, e4)
  a0, a1 = 0.5 * np.linalg.norm(np.cross(e0, e1)), 0.5 * np.linalg.norm(np.cross(e0, e2))
  c = np.array([c03 + c04, c01 + c02, -(c01 + c03), -(c02 + c04)])
  return (np.outer(c, c) * mu * thickness**3 / (8.0 * (a0 + a1))).reshape(-1)


def _read_mesh_file(path):
  """(vertices (n, 3) float64, triangles (t, 3) int64) of a binary / ASCII STL or an OBJ file."""
  ext = os.path.splitext(path)[1].lower()
  with open(path, "rb") as fh:
    buf = fh.read()
  if ext == ".stl":
    if buf[:5] == b"solid" and b"facet" in buf[:1024]:  # ASCII STL
      vals = [ln.split()[1:4] for ln in buf.decode("ascii", "replace").splitlines() if ln.strip().startswith("vertex")]
      v = np.array(vals, dtype=np.float64)
    else:
      n = int(np.frombuffer(buf, dtype="<u4", count=1, offset=80)[0])
      rec = np.dtype([("n", "<f4", 3), ("v", "<f4", 9), ("a", "<u2")])
      v = np.frombuffer(buf, dtype=rec, count=n, offset=84)["v"].reshape(-1, 3).astype(np.float64)
    return v, np.arange(len(v)).reshape(-1, 3)
  if ext == ".obj":
    verts, faces = [], []
    for ln in buf.decode("utf-8", "replace").splitlines():
      p = ln.split()
      if not p:
        continue
      if p[0] == "v":
        verts.append([float(x) for x in p[1:4]])
      elif p[0] == "f":
        idx = [int(t.split("/")[0]) for t in p[1:]]
        idx = [i - 1 if i > 0 else len(verts) + i for i in idx]
        for k in range(1, len(idx) - 1):  # fan triangulation
          faces.append([idx[0], idx[k], idx[k + 1]])
    return np.array(verts, dtype=np.float64).reshape(-1, 3), np.array(faces, dtype=np.int64).reshape(-1, 3)
  raise NotImplementedError(f"mesh file type '{ext}' is not supported (STL / OBJ only)")


def _mesh_mass_props(v, f):
  """(volume, COM, inertia about the COM at unit density) of a closed triangle mesh from signed
  tetrahedra against the origin (MuJoCo's exact-volume mesh inertia; |volume| so that inverted
  winding still gives a positive mass)."""
  if len(f) == 0:
    return 0.0, np.zeros(3), np.zeros((3, 3))
  a, b, c = v[f[:, 0]], v[f[:, 1]], v[f[:, 2]]
  dv = np.einsum("ij,ij->i", a, np.cross(b, c)) / 6.0
  vol = dv.sum()
  if abs(vol) < 1e-300:
    return 0.0, np.zeros(3), np.zeros((3, 3))
  com = (dv[:, None] * (a + b + c) / 4.0).sum(axis=0) / vol
  # second moments of each tetrahedron (origin, a, b, c): dv/20 (sum_i x_i x_i^T + s s^T), s = a+b+c
  s = a + b + c
  C = (dv[:, None, None] / 20.0 * (np.einsum("ij,ik->ijk", a, a) + np.einsum("ij,ik->ijk", b, b) + np.einsum("ij,ik->ijk", c, c)
                                   + np.einsum("ij,ik->ijk", s, s))).sum(axis=0)
  C = C - vol * np.outer(com, com)  # covariance about the COM
  I = np.trace(C) * np.eye(3) - C
  sign = 1.0 if vol > 0 else -1.0
  return abs(vol), com, sign * I


NFLUID = 12  # mjNFLUID: (interaction coef, blunt / slender / angular drag, Kutta / Magnus lift, virtual mass x3, virtual inertia x3)


def fluid_semiaxes(gtype, size):
  """Semi-axes of the ellipsoid that stands in for a geom in the fluid model (passive.py:42-59)."""
  if gtype == GeomType.SPHERE:
    return np.array([size[0]] * 3)
  if gtype == GeomType.CAPSULE:
    return np.array([size[0], size[0], size[1] + size[0]])
  if gtype == GeomType.CYLINDER:
    return np.array([size[0], size[0], size[1]])
  return np.asarray(size[:3], dtype=float)


def added_mass_kappa(dx, dy, dz):
  """kappa_x = dx dy dz * int_0^inf dl / ((dx^2 + l)^1.5 sqrt((dy^2 + l)(dz^2 + l))) of an ellipsoid (the
  potential-flow added-mass integral MuJoCo's compiler evaluates for fluidshape="ellipsoid"), here in closed
  form through Carlson's symmetric integral: (2/3) dx dy dz R_D(dy^2, dz^2, dx^2).  kx + ky + kz = 2."""
  from scipy.special import elliprd

  return 2.0 / 3.0 * dx * dy * dz * float(elliprd(dy * dy, dz * dz, dx * dx))


def _geom_fluid(ga, gtype, size):
  """geom_fluid row (types.py:961, read by passive.py:335-450): zero unless fluidshape="ellipsoid"; then
  (1, fluidcoef[5], virtual mass[3], virtual inertia[3]) per unit fluid density.  Virtual mass
  m_i = V k_i / (2 - k_i) and inertia I_x = V / 5 (dy^2 - dz^2)^2 |kz - ky| / |2 (dy^2 - dz^2) + (dy^2 + dz^2)(ky - kz)|
  (cyclic), the ellipsoid's potential-flow added mass (MuJoCo's fluid model documentation)."""
  out = np.zeros(NFLUID)
  if ga.get("fluidshape", "none") != "ellipsoid":
    return out
  out[0] = 1.0
  out[1:6] = _merge_vec([0.5, 0.25, 1.5, 1.0, 1.0], _floats(ga["fluidcoef"]) if "fluidcoef" in ga else [])
  d = fluid_semiaxes(gtype, size)
  k = [added_mass_kappa(d[i], d[(i + 1) % 3], d[(i + 2) % 3]) for i in range(3)]
  vol = 4.0 / 3.0 * math.pi * d[0] * d[1] * d[2]
  for i in range(3):
    out[6 + i] = vol * k[i] / max(MJ_MINVAL, 2.0 - k[i])
    j, l = (i + 1) % 3, (i + 2) % 3
    dj2, dl2 = d[j] ** 2, d[l] ** 2
    num = (dj2 - dl2) ** 2 * abs(k[l] - k[j])
    den = abs(2.0 * (dj2 - dl2) + (dj2 + dl2) * (k[j] - k[l]))
    out[9 + i] = vol / 5.0 * num / max(MJ_MINVAL, den)
  return out


def _geom_inertia(gtype, size, mass):
  """Principal moments of a solid geom of the given mass (MuJoCo mjCGeom inertia)."""
  r = size[0]
  if gtype == GeomType.SPHERE:
    i = 2.0 * mass * r * r / 5.0
    return np.array([i, i, i])
  if gtype == GeomType.CAPSULE:
    h = 2.0 * size[1]
    sphere_mass = mass * 4.0 * r / (4.0 * r + 3.0 * h)
    cyl_mass = mass - sphere_mass
    i0 = cyl_mass * (3 * r * r + h * h) / 12.0
    i2 = cyl_mass * r * r / 2.0
    sph = 2.0 * sphere_mass * r * r / 5.0
    i0 += sph + sphere_mass * h * (3 * r + 2 * h) / 8.0
    i2 += sph
    return np.array([i0, i0, i2])
  if gtype == GeomType.CYLINDER:
    h = 2.0 * size[1]
    i0 = mass * (3 * r * r + h * h) / 12.0
    return np.array([i0, i0, mass * r * r / 2.0])
  if gtype == GeomType.BOX:
    s = size
    return np.array([mass * (s[1] ** 2 + s[2] ** 2) / 3.0, mass * (s[0] ** 2 + s[2] ** 2) / 3.0, mass * (s[0] ** 2 + s[1] ** 2) / 3.0])
  if gtype == GeomType.ELLIPSOID:
    s = size
    return np.array([mass * (s[1] ** 2 + s[2] ** 2) / 5.0, mass * (s[0] ** 2 + s[2] ** 2) / 5.0, mass * (s[0] ** 2 + s[1] ** 2) / 5.0])
  return np.zeros(3)


def _eig3(I):
  """Symmetric 3x3 eigendecomposition, eigenvalues descending, right-handed eigenvector frame."""
  w, V = np.linalg.eigh(I)
  order = np.argsort(-w)
  w, V = w[order], V[:, order]
  if np.linalg.det(V) < 0:
    V[:, 2] = -V[:, 2]
  return w, V


# ---------------------------------------------------------------------------------------------
# set_const: qpos0-dependent constants (reference io.py:2222-2407), fp64 host restatement
# ---------------------------------------------------------------------------------------------


def _kinematics_qpos0(m: MjModel, qpos=None):
  """Forward kinematics + subtree com + cdof + composite inertia + dense qM at qpos0 (fp64)."""
  nb, nv = m.nbody, m.nv
  qpos = m.qpos0 if qpos is None else np.asarray(qpos, float)
  xpos = np.zeros((nb, 3))
  xquat = np.tile([1.0, 0, 0, 0], (nb, 1)).astype(float)
  xanchor = np.zeros((m.njnt, 3))
  xaxis = np.zeros((m.njnt, 3))
  for b in range(1, nb):
    p = m.body_parentid[b]
    ja, jn = m.body_jntadr[b], m.body_jntnum[b]
    if jn == 1 and m.jnt_type[ja] == JointType.FREE:
      a = m.jnt_qposadr[ja]
      xpos[b] = qpos[a : a + 3]
      q = qpos[a + 3 : a + 7]
      xquat[b] = q / np.linalg.norm(q)
      xanchor[ja] = xpos[b]
      xaxis[ja] = m.jnt_axis[ja]
      continue
    pos = rot_vec(xquat[p], m.body_pos[b]) + xpos[p]
    quat = quat_mul(xquat[p], m.body_quat[b])
    for j in range(ja, ja + jn) if jn else []:
      a = m.jnt_qposadr[j]
      xanchor[j] = rot_vec(quat, m.jnt_pos[j]) + pos
      xaxis[j] = rot_vec(quat, m.jnt_axis[j])
      t = m.jnt_type[j]
      if t == JointType.BALL:
        ql = qpos[a : a + 4] / np.linalg.norm(qpos[a : a + 4])
        quat = quat_mul(quat, ql)
        pos = xanchor[j] - rot_vec(quat, m.jnt_pos[j])
      elif t == JointType.SLIDE:
        pos = pos + xaxis[j] * (qpos[a] - m.qpos0[a])
      elif t == JointType.HINGE:
        ang = qpos[a] - m.qpos0[a]
        ql = np.array([math.cos(ang / 2), *(m.jnt_axis[j] * math.sin(ang / 2))])
        quat = quat_mul(quat, ql)
        pos = xanchor[j] - rot_vec(quat, m.jnt_pos[j])
    xpos[b] = pos
    xquat[b] = quat / np.linalg.norm(quat)
  xmat = np.array([quat_to_mat(q) for q in xquat])
  xipos = np.array([xpos[b] + rot_vec(xquat[b], m.body_ipos[b]) for b in range(nb)])
  ximat = np.array([quat_to_mat(quat_mul(xquat[b], m.body_iquat[b])) for b in range(nb)])
  # subtree com
  st = xipos * m.body_mass[:, None]
  for b in range(nb - 1, 0, -1):
    st[m.body_parentid[b]] += st[b]
  subtree_com = np.zeros((nb, 3))
  for b in range(nb):
    if m.body_subtreemass[b] != 0:
      subtree_com[b] = st[b] / m.body_subtreemass[b]
  # cinert (6x6 spatial inertia about subtree com of root), cdof
  cinert = np.zeros((nb, 6, 6))
  for b in range(1, nb):
    R = ximat[b]
    Ib = R @ np.diag(m.body_inertia[b]) @ R.T
    d = xipos[b] - subtree_com[m.body_rootid[b]]
    mass = m.body_mass[b]
    cd = _skew(d)
    cinert[b, :3, :3] = Ib - mass * cd @ cd
    cinert[b, :3, 3:] = mass * cd
    cinert[b, 3:, :3] = -mass * cd
    cinert[b, 3:, 3:] = mass * np.eye(3)
  cdof = np.zeros((nv, 6))
  for j in range(m.njnt):
    b = m.jnt_bodyid[j]
    da = m.jnt_dofadr[j]
    off = subtree_com[m.body_rootid[b]] - xanchor[j]
    t = m.jnt_type[j]
    if t == JointType.FREE:
      cdof[da : da + 3, 3:] = np.eye(3)
      for k in range(3):
        ax = xmat[b][:, k]
        cdof[da + 3 + k] = np.concatenate([ax, np.cross(ax, off)])
    elif t == JointType.BALL:
      for k in range(3):
        ax = xmat[b][:, k]
        cdof[da + k] = np.concatenate([ax, np.cross(ax, off)])
    elif t == JointType.SLIDE:
      cdof[da] = np.concatenate([np.zeros(3), xaxis[j]])
    else:
      cdof[da] = np.concatenate([xaxis[j], np.cross(xaxis[j], off)])
  crb = cinert.copy()
  for b in range(nb - 1, 0, -1):
    p = m.body_parentid[b]
    if p > 0:
      crb[p] += crb[b]
  M = np.zeros((nv, nv))
  for i in range(nv):
    buf = crb[m.dof_bodyid[i]] @ cdof[i]
    j = i
    while j >= 0:
      M[i, j] += cdof[j] @ buf
      j = m.dof_parentid[j]
    M[i, i] += m.dof_armature[i]
  M = np.tril(M) + np.tril(M, -1).T
  return dict(xpos=xpos, xquat=xquat, xmat=xmat, xipos=xipos, subtree_com=subtree_com, cdof=cdof, M=M)


def _spatial_tendon_qpos0(m: MjModel, k: dict, t: int):
  """Length and Jacobian of spatial tendon t at qpos0 (tendon_geom.py restates smooth.py:3172-3465)."""
  from .tendon_geom import tendon_length_jac

  xpos, xquat = k["xpos"], k["xquat"]
  site_xpos = np.array([xpos[b] + rot_vec(xquat[b], m.site_pos[s]) for s, b in enumerate(m.site_bodyid)]).reshape(-1, 3)
  geom_xpos = np.array([xpos[b] + rot_vec(xquat[b], m.geom_pos[g]) for g, b in enumerate(m.geom_bodyid)]).reshape(-1, 3)
  geom_xmat = np.array([quat_to_mat(quat_mul(xquat[b], m.geom_quat[g])) for g, b in enumerate(m.geom_bodyid)]).reshape(-1, 3, 3)

  def jac_point(p, b):
    J = np.zeros((3, m.nv))
    off = p - k["subtree_com"][m.body_rootid[b]]
    while b > 0:
      for d in range(m.body_dofadr[b], m.body_dofadr[b] + m.body_dofnum[b]):
        J[:, d] = k["cdof"][d, 3:] + np.cross(k["cdof"][d, :3], off)
      b = m.body_parentid[b]
    return J

  return tendon_length_jac(m, t, site_xpos, m.site_bodyid, geom_xpos, geom_xmat, jac_point)


def _site_moment(m: MjModel, k: dict, a: int):
  """Moment row of a SITE / SLIDERCRANK transmission at the pose of `k` (smooth.py:2150-2241, 2274-2442; the
  oracle's site_transmission restates the same)."""
  xpos, xquat = k["xpos"], k["xquat"]
  sx = lambda s_: xpos[m.site_bodyid[s_]] + rot_vec(xquat[m.site_bodyid[s_]], m.site_pos[s_])
  sm = lambda s_: quat_to_mat(quat_mul(xquat[m.site_bodyid[s_]], m.site_quat[s_]))

  def jac(p, b, dof):
    db = m.dof_bodyid[dof]
    bb, ok = b, db == 0
    while bb != 0 and not ok:
      ok = bb == db
      bb = m.body_parentid[bb]
    if not ok:
      return np.zeros(3), np.zeros(3)
    cd = k["cdof"][dof]
    return cd[3:] + np.cross(cd[:3], p - k["subtree_com"][m.body_rootid[b]]), cd[:3].copy()

  def last(b):
    return m.body_dofadr[b] + m.body_dofnum[b] - 1 if b > 0 else -1

  gear = m.actuator_gear[a]
  i1, i2 = m.actuator_trnid[a]
  mom = np.zeros(m.nv)
  if m.actuator_trntype[a] == TrnType.SLIDERCRANK:
    rod = m.actuator_cranklength[a]
    axis = sm(i2)[:, 2]
    vec = sx(i1) - sx(i2)
    av = vec @ axis
    det = av * av + rod * rod - vec @ vec
    if det > 0:
      sdet = np.sqrt(det)
      sc = 1 - av / sdet
      dldv, dlda = axis * sc + vec / sdet, vec * sc
    else:
      dldv, dlda = axis, vec
    d1, d2 = last(m.body_weldid[m.site_bodyid[i1]]), last(m.body_weldid[m.site_bodyid[i2]])
    while d1 >= 0 or d2 >= 0:
      da = max(d1, d2)
      jp2, jr2 = jac(sx(i2), m.site_bodyid[i2], da)
      jp1, _ = jac(sx(i1), m.site_bodyid[i1], da)
      mom[da] = (dlda @ np.cross(jr2, axis) + dldv @ (jp1 - jp2)) * gear[0]
      if d1 == da:
        d1 = m.dof_parentid[d1]
      if d2 == da:
        d2 = m.dof_parentid[d2]
    return mom
  if i2 < 0:
    R = sm(i1)
    da = last(m.body_weldid[m.site_bodyid[i1]])
    while da >= 0:
      jp, jr = jac(sx(i1), m.site_bodyid[i1], da)
      mom[da] = jp @ (R @ gear[:3]) + jr @ (R @ gear[3:])
      da = m.dof_parentid[da]
    return mom
  R = sm(i2)
  d1, d2 = last(m.body_weldid[m.site_bodyid[i1]]), last(m.body_weldid[m.site_bodyid[i2]])
  while d1 >= 0 or d2 >= 0:
    da = max(d1, d2)
    if d1 == da and d2 == da:
      break
    jp, jr = jac(sx(i1), m.site_bodyid[i1], da)
    jq, jqr = jac(sx(i2), m.site_bodyid[i2], da)
    mom[da] = (jp - jq) @ (R @ gear[:3]) + (jr - jqr) @ (R @ gear[3:])
    if d1 == da:
      d1 = m.dof_parentid[d1]
    if d2 == da:
      d2 = m.dof_parentid[d2]
  return mom


def _skew(v):
  return np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]])


def set_const(m: MjModel):
  """Compute qpos0-dependent constants exactly as io.set_const_0 (io.py:2222-2407) does."""
  nv, nb = m.nv, m.nbody
  k = _kinematics_qpos0(m)
  M = k["M"]
  # fixed tendons at qpos0: length0, the dense Jacobians, armature in M (smooth.py:916-1000)
  nt = getattr(m, "ntendon", 0)
  tenJ = np.zeros((nt, nv))
  m.tendon_length0 = np.zeros(nt)
  for t in range(nt):
    if m.wrap_type[m.tendon_adr[t]] != WrapType.JOINT:
      m.tendon_length0[t], tenJ[t] = _spatial_tendon_qpos0(m, k, t)
    else:
      for w in range(m.tendon_adr[t], m.tendon_adr[t] + m.tendon_num[t]):
        j = m.wrap_objid[w]
        m.tendon_length0[t] += m.wrap_prm[w] * m.qpos0[m.jnt_qposadr[j]]
        tenJ[t, m.jnt_dofadr[j]] += m.wrap_prm[w]
    if m.tendon_armature[t]:
      M = M + m.tendon_armature[t] * np.outer(tenJ[t], tenJ[t])
  if nt:
    # springlength -1: the spring rests at the qpos0 length (MuJoCo's compiler)
    ls = m.tendon_lengthspring
    for t in range(nt):
      if ls[t, 0] == -1 and ls[t, 1] == -1:
        ls[t] = m.tendon_length0[t]
  m.stat.meaninertia = float(np.trace(M) / nv) if nv else 1.0
  Minv = np.linalg.inv(M) if nv else np.zeros((0, 0))
  # dof_invweight0 (io.py:1802-1843)
  diag = np.diag(Minv) if nv else np.zeros(0)
  inv = np.zeros(nv)
  for i in range(nv):
    j = m.dof_jntid[i]
    t, da = m.jnt_type[j], m.jnt_dofadr[j]
    if t == JointType.FREE:
      inv[i] = diag[da : da + 3].mean() if i < da + 3 else diag[da + 3 : da + 6].mean()
    elif t == JointType.BALL:
      inv[i] = diag[da : da + 3].mean()
    else:
      inv[i] = diag[i]
  m.dof_invweight0 = inv
  # tendon_invweight0 = J M^-1 J' at qpos0
  m.tendon_invweight0 = np.array([tenJ[t] @ Minv @ tenJ[t] for t in range(nt)]) if nt else np.zeros(0)
  # body_invweight0 (io.py:1846-1956)
  biw = np.zeros((nb, 2))
  for b in range(1, nb):
    if m.body_weldid[b] == 0 or nv == 0:
      continue
    bb = b
    while bb > 0 and m.body_dofnum[bb] == 0:
      bb = m.body_parentid[bb]
    if bb == 0:
      continue
    off = k["xipos"][b] - k["subtree_com"][m.body_rootid[b]]
    J = np.zeros((6, nv))
    d = m.body_dofadr[bb] + m.body_dofnum[bb] - 1
    while d >= 0:
      ang, lin = k["cdof"][d, :3], k["cdof"][d, 3:]
      J[:3, d] = lin + np.cross(ang, off)
      J[3:, d] = ang
      d = m.dof_parentid[d]
    cols = np.nonzero(np.any(J != 0, axis=0))[0]
    A = J[:, cols] @ Minv[np.ix_(cols, cols)] @ J[:, cols].T
    tr, rot = np.trace(A[:3, :3]) / 3.0, np.trace(A[3:, 3:]) / 3.0
    if tr < MJ_MINVAL and rot > MJ_MINVAL:
      tr = rot
    elif rot < MJ_MINVAL and tr > MJ_MINVAL:
      rot = tr
    biw[b] = [tr, rot]
  m.body_invweight0 = biw
  # connect / weld offsets at qpos0 (MuJoCo's compiler; the reference reads them from eq_data,
  # constraint.py:199-209, 855-866): connect anchor2 = body2-frame image of body1's anchor; weld
  # relpose (when its quaternion is zero) = body1-frame pose of body2's anchor and orientation
  for e in range(getattr(m, "neq", 0)):
    if m.eq_objtype[e] != ObjType.BODY or m.eq_type[e] not in (EqType.CONNECT, EqType.WELD):
      continue
    b1, b2, dat = m.eq_obj1id[e], m.eq_obj2id[e], m.eq_data[e]
    R1, R2 = quat_to_mat(k["xquat"][b1]), quat_to_mat(k["xquat"][b2])
    if m.eq_type[e] == EqType.CONNECT:
      p = k["xpos"][b1] + R1 @ dat[:3]
      dat[3:6] = R2.T @ (p - k["xpos"][b2])
    elif not np.any(dat[6:10]):
      p = k["xpos"][b2] + R2 @ dat[:3]
      dat[3:6] = R1.T @ (p - k["xpos"][b1])
      q1 = k["xquat"][b1]
      dat[6:10] = quat_mul(np.array([q1[0], -q1[1], -q1[2], -q1[3]]), k["xquat"][b2])
  # cameras / lights at qpos0 (fixed-frame placement), io.py:2005-2053
  xpos, xquat, sc = k["xpos"], k["xquat"], k["subtree_com"]
  m.cam_pos0 = np.zeros((m.ncam, 3))
  m.cam_poscom0 = np.zeros((m.ncam, 3))
  m.cam_mat0 = np.zeros((m.ncam, 9))
  for c in range(m.ncam):
    b = m.cam_bodyid[c]
    cx = xpos[b] + rot_vec(xquat[b], m.cam_pos[c])
    cm = quat_to_mat(quat_mul(xquat[b], m.cam_quat[c]))
    m.cam_pos0[c] = cx - xpos[b]
    t = m.cam_targetbodyid[c]
    m.cam_poscom0[c] = cx - sc[t if t >= 0 else b]
    m.cam_mat0[c] = cm.reshape(-1)
  m.light_pos0 = np.zeros((m.nlight, 3))
  m.light_poscom0 = np.zeros((m.nlight, 3))
  m.light_dir0 = np.zeros((m.nlight, 3))
  for l in range(m.nlight):
    b = m.light_bodyid[l]
    lx = xpos[b] + rot_vec(xquat[b], m.light_pos[l])
    ld = rot_vec(xquat[b], m.light_dir[l])
    m.light_pos0[l] = lx - xpos[b]
    t = m.light_targetbodyid[l]
    m.light_poscom0[l] = lx - sc[t if t >= 0 else b]
    m.light_dir0[l] = ld
  # actuator_acc0 = ||M^-1 moment|| (io.py:2367-2380); joint transmissions only
  acc0 = np.zeros(m.nu)
  for a in range(m.nu):
    vec = np.zeros(nv)
    j = m.actuator_trnid[a, 0]
    if m.actuator_trntype[a] == TrnType.TENDON:
      acc0[a] = np.linalg.norm(Minv @ (m.actuator_gear[a, 0] * tenJ[j]))
      continue
    if m.actuator_trntype[a] in (TrnType.SITE, TrnType.SLIDERCRANK, TrnType.BODY):
      acc0[a] = np.linalg.norm(Minv @ _site_moment(m, k, a)) if m.actuator_trntype[a] != TrnType.BODY else 0.0
      continue
    t = m.jnt_type[j]
    da = m.jnt_dofadr[j]
    if t == JointType.FREE:
      vec[da : da + 6] = m.actuator_gear[a]
    elif t == JointType.BALL:
      vec[da : da + 3] = m.actuator_gear[a, :3]
    else:
      vec[da] = m.actuator_gear[a, 0]
    acc0[a] = np.linalg.norm(Minv @ vec)
  m.actuator_acc0 = acc0


def _mesh_polygons(v):
  """Polygons of the convex hull of mesh vertices `v` (MuJoCo's mesh_poly* data): the hull's coplanar
  triangles merged into one face each.  Returns (loops, normals, polymap): per polygon its vertex loop (mesh
  vertex ids, counter-clockwise about the outward normal, starting at its smallest id), its outward unit
  normal, and per vertex the polygons that contain it (ascending).  Polygons are ordered by their smallest
  vertex id, then their loop.  Vertices off the hull map to no polygon."""
  n = len(v)
  if n < 4:
    return [], np.zeros((0, 3)), [[] for _ in range(n)]
  from scipy.spatial import ConvexHull

  h = ConvexHull(v)
  scale = max(float(np.abs(v).max()), 1e-12)
  groups = []  # (normal, offset, triangles)
  for tri, eq in zip(h.simplices, h.equations):
    nrm, off = eq[:3], eq[3]
    for g in groups:
      if np.dot(g[0], nrm) > 1.0 - 1e-9 and abs(g[1] - off) < 1e-9 * scale:
        g[2].append(tri)
        break
    else:
      groups.append((nrm, off, [tri]))
  polys = []
  for nrm, _, tris in groups:
    edges = {}
    for a, b, c in tris:
      if np.dot(np.cross(v[b] - v[a], v[c] - v[a]), nrm) < 0:
        b, c = c, b
      for e0, e1 in ((a, b), (b, c), (c, a)):
        edges[(int(e0), int(e1))] = True
    nxt = {e0: e1 for (e0, e1) in edges if (e1, e0) not in edges}  # boundary, counter-clockwise
    start = min(nxt)
    loop = [start]
    while nxt[loop[-1]] != start and len(loop) <= len(nxt):
      loop.append(nxt[loop[-1]])
    polys.append((loop, nrm / np.linalg.norm(nrm)))
  polys.sort(key=lambda p: (min(p[0]), p[0]))
  pmap = [[] for _ in range(n)]
  for k, (loop, _) in enumerate(polys):
    for i in loop:
      pmap[i].append(k)
  return [p[0] for p in polys], np.array([p[1] for p in polys]).reshape(-1, 3), pmap


def _hull_faces(v):
  """Outward-oriented triangles of the convex hull of `v` (inline meshes without faces).  Needs scipy
  (an optional dependency of the compiler, used only for this case)."""
  try:
    from scipy.spatial import ConvexHull
  except ImportError as e:  # pragma: no cover - scipy is installed in this image
    raise ImportError("an inline <mesh vertex=...> without faces needs scipy.spatial.ConvexHull") from e

  h = ConvexHull(v)
  c = v.mean(axis=0)
  f = h.simplices.astype(np.int64).copy()
  for k, (i, j, l) in enumerate(f):
    if np.dot(np.cross(v[j] - v[i], v[l] - v[i]), v[i] - c) < 0:
      f[k] = (i, l, j)
  return f


def load_model_from_string(xml: str, basedir: str = ".") -> MjModel:
  return _Compiler(ET.fromstring(xml), basedir).compile()


def load_model(path: str) -> MjModel:
  """Compile an MJCF file (analogue of `mujoco.MjModel.from_xml_path`)."""
  root = ET.parse(path).getroot()
  return _Compiler(root, os.path.dirname(os.path.abspath(path))).compile()


def is_sparse(m) -> bool:
  """Dense/sparse switch of the reference (io.py:67-74)."""
  if m.opt.jacobian == JacobianType.AUTO:
    return m.nv > 32
  return m.opt.jacobian == JacobianType.SPARSE
