"""Enums, constants and the Model / Data containers of the MI355X stepper.

Mirrors the public type surface of mujoco_warp (`mujoco_warp/_src/types.py`):
enum names/values (`types.py:74-638`), the `Option` (`:706-772`), `Statistic`
(`:776`), `Model` (`:833-1603`), `Contact` (`:1617-1655`), `Constraint`
(`:1658-1699`) and `Data` (`:1702-1896`) dataclasses.  Array fields are
`torch.Tensor`s on the ROCm device instead of `wp.array`s.  Batched model
fields (`"*"` leading dim in the reference) keep the reference semantics: the
leading dimension is 1 or nworld and is indexed `worldid % shape[0]`.
"""

from __future__ import annotations

import dataclasses
import enum
from typing import Any, Callable, Optional

MJ_MINVAL = 1e-15
MJ_MAXVAL = 1e10
MJ_MINIMP = 0.0001
MJ_MAXIMP = 0.9999
MJ_MAXCONPAIR = 50
MJ_MINMU = 1e-5

TILE_SIZE_JTDAJ_SPARSE = 16
TILE_SIZE_JTDAJ_DENSE = 16


class BroadphaseType(enum.IntEnum):
  NXN = 0
  SAP_TILE = 1
  SAP_SEGMENTED = 2


class BroadphaseFilter(enum.IntFlag):
  PLANE = 1
  SPHERE = 2
  AABB = 4
  OBB = 8


class CamLightType(enum.IntEnum):
  FIXED = 0
  TRACK = 1
  TRACKCOM = 2
  TARGETBODY = 3
  TARGETBODYCOM = 4


class DisableBit(enum.IntFlag):
  CONSTRAINT = 1 << 0
  EQUALITY = 1 << 1
  FRICTIONLOSS = 1 << 2
  LIMIT = 1 << 3
  CONTACT = 1 << 4
  SPRING = 1 << 5
  DAMPER = 1 << 6
  GRAVITY = 1 << 7
  CLAMPCTRL = 1 << 8
  WARMSTART = 1 << 9
  FILTERPARENT = 1 << 10
  ACTUATION = 1 << 11
  REFSAFE = 1 << 12
  SENSOR = 1 << 13
  MIDPHASE = 1 << 14
  EULERDAMP = 1 << 15
  AUTORESET = 1 << 16
  NATIVECCD = 1 << 17
  ISLAND = 1 << 18


class EnableBit(enum.IntFlag):
  OVERRIDE = 1 << 0
  ENERGY = 1 << 1
  FWDINV = 1 << 2
  INVDISCRETE = 1 << 3
  MULTICCD = 1 << 4


class TrnType(enum.IntEnum):
  JOINT = 0
  JOINTINPARENT = 1
  SLIDERCRANK = 2
  TENDON = 3
  SITE = 4
  BODY = 5


class DynType(enum.IntEnum):
  NONE = 0
  INTEGRATOR = 1
  FILTER = 2
  FILTEREXACT = 3
  MUSCLE = 4
  USER = 5


class GainType(enum.IntEnum):
  FIXED = 0
  AFFINE = 1
  MUSCLE = 2
  USER = 3


class BiasType(enum.IntEnum):
  NONE = 0
  AFFINE = 1
  MUSCLE = 2
  USER = 3


class WrapType(enum.IntEnum):
  """Tendon wrap object (types.py:580-595, MuJoCo mjtWrap)."""
  NONE = 0
  JOINT = 1
  PULLEY = 2
  SITE = 3
  SPHERE = 4
  CYLINDER = 5


class JointType(enum.IntEnum):
  FREE = 0
  BALL = 1
  SLIDE = 2
  HINGE = 3


class ConeType(enum.IntEnum):
  PYRAMIDAL = 0
  ELLIPTIC = 1


class IntegratorType(enum.IntEnum):
  EULER = 0
  RK4 = 1
  IMPLICIT = 2
  IMPLICITFAST = 3


class GeomType(enum.IntEnum):
  PLANE = 0
  HFIELD = 1
  SPHERE = 2
  CAPSULE = 3
  ELLIPSOID = 4
  CYLINDER = 5
  BOX = 6
  MESH = 7
  SDF = 8


class SolverType(enum.IntEnum):
  PGS = 0
  CG = 1
  NEWTON = 2


class JacobianType(enum.IntEnum):
  DENSE = 0
  SPARSE = 1
  AUTO = 2


class ConstraintState(enum.IntEnum):
  SATISFIED = 0
  QUADRATIC = 1
  LINEARNEG = 2
  LINEARPOS = 3
  CONE = 4


class ConstraintType(enum.IntEnum):
  EQUALITY = 0
  FRICTION_DOF = 1
  FRICTION_TENDON = 2
  LIMIT_JOINT = 3
  LIMIT_TENDON = 4
  CONTACT_FRICTIONLESS = 5
  CONTACT_PYRAMIDAL = 6
  CONTACT_ELLIPTIC = 7


class ContactType(enum.IntFlag):
  CONSTRAINT = 1
  SENSOR = 2


class ObjType(enum.IntEnum):
  UNKNOWN = 0
  BODY = 1
  XBODY = 2
  JOINT = 3
  DOF = 4
  GEOM = 5
  SITE = 6
  CAMERA = 7
  LIGHT = 8
  FLEX = 9
  MESH = 10
  TENDON = 18
  ACTUATOR = 19


class SensorType(enum.IntEnum):
  """mjtSensor (types.py:466-524 takes the values from mujoco.mjtSensor; restated from MuJoCo's
  mjmodel.h since `mujoco` is not importable here)."""

  TOUCH = 0
  ACCELEROMETER = 1
  VELOCIMETER = 2
  GYRO = 3
  FORCE = 4
  TORQUE = 5
  MAGNETOMETER = 6
  RANGEFINDER = 7
  CAMPROJECTION = 8
  JOINTPOS = 9
  JOINTVEL = 10
  TENDONPOS = 11
  TENDONVEL = 12
  ACTUATORPOS = 13
  ACTUATORVEL = 14
  ACTUATORFRC = 15
  JOINTACTFRC = 16
  TENDONACTFRC = 17
  BALLQUAT = 18
  BALLANGVEL = 19
  JOINTLIMITPOS = 20
  JOINTLIMITVEL = 21
  JOINTLIMITFRC = 22
  TENDONLIMITPOS = 23
  TENDONLIMITVEL = 24
  TENDONLIMITFRC = 25
  FRAMEPOS = 26
  FRAMEQUAT = 27
  FRAMEXAXIS = 28
  FRAMEYAXIS = 29
  FRAMEZAXIS = 30
  FRAMELINVEL = 31
  FRAMEANGVEL = 32
  FRAMELINACC = 33
  FRAMEANGACC = 34
  SUBTREECOM = 35
  SUBTREELINVEL = 36
  SUBTREEANGMOM = 37
  INSIDESITE = 38
  GEOMDIST = 39
  GEOMNORMAL = 40
  GEOMFROMTO = 41
  CONTACT = 42
  E_POTENTIAL = 43
  E_KINETIC = 44
  CLOCK = 45  # after INSIDESITE, GEOMDIST, GEOMNORMAL, GEOMFROMTO, CONTACT, E_POTENTIAL, E_KINETIC
  TACTILE = 46  # this build's value (MuJoCo's enum position unpinned: mujoco is not importable here)


class DataType(enum.IntEnum):
  """mjtDataType (types.py:158-166)."""

  REAL = 0
  POSITIVE = 1
  AXIS = 2
  QUATERNION = 3


class Stage(enum.IntEnum):
  """mjtStage (types.py:530-540)."""

  NONE = 0
  POS = 1
  VEL = 2
  ACC = 3


# sensors built on the device path (sensor.py:459-706, 1251-1373, 1697-1997 subset)
SUPPORTED_SENSORS = {
  SensorType.ACCELEROMETER, SensorType.VELOCIMETER, SensorType.GYRO, SensorType.FORCE, SensorType.TORQUE,
  SensorType.MAGNETOMETER, SensorType.JOINTPOS, SensorType.JOINTVEL, SensorType.ACTUATORPOS, SensorType.ACTUATORVEL,
  SensorType.ACTUATORFRC, SensorType.JOINTACTFRC, SensorType.BALLQUAT, SensorType.BALLANGVEL, SensorType.FRAMEPOS,
  SensorType.FRAMEQUAT, SensorType.FRAMEXAXIS, SensorType.FRAMEYAXIS, SensorType.FRAMEZAXIS, SensorType.FRAMELINVEL,
  SensorType.FRAMEANGVEL, SensorType.FRAMELINACC, SensorType.FRAMEANGACC, SensorType.SUBTREECOM, SensorType.CLOCK,
  SensorType.TOUCH, SensorType.TENDONPOS, SensorType.TENDONVEL, SensorType.TENDONACTFRC, SensorType.JOINTLIMITPOS,
  SensorType.JOINTLIMITVEL, SensorType.JOINTLIMITFRC, SensorType.TENDONLIMITPOS, SensorType.TENDONLIMITVEL,
  SensorType.TENDONLIMITFRC, SensorType.SUBTREELINVEL, SensorType.SUBTREEANGMOM, SensorType.E_POTENTIAL, SensorType.E_KINETIC,
  SensorType.GEOMDIST, SensorType.GEOMNORMAL, SensorType.GEOMFROMTO, SensorType.INSIDESITE, SensorType.CAMPROJECTION,
  SensorType.CONTACT, SensorType.TACTILE,
}
# sensors that need rne_postconstraint (io.py:542-551)
RNE_POSTCONSTRAINT_SENSORS = {
  SensorType.ACCELEROMETER, SensorType.FORCE, SensorType.TORQUE, SensorType.FRAMELINACC, SensorType.FRAMEANGACC,
}


class EqType(enum.IntEnum):
  CONNECT = 0
  WELD = 1
  JOINT = 2
  TENDON = 3
  FLEX = 4


class State(enum.IntFlag):
  """mjtState bitflags used by get_state / set_state (types.py:598-638)."""

  TIME = 1 << 0
  QPOS = 1 << 1
  QVEL = 1 << 2
  ACT = 1 << 3
  WARMSTART = 1 << 4
  CTRL = 1 << 5
  QFRC_APPLIED = 1 << 6
  XFRC_APPLIED = 1 << 7
  EQ_ACTIVE = 1 << 8
  MOCAP_POS = 1 << 9
  MOCAP_QUAT = 1 << 10
  USERDATA = 1 << 11
  PLUGIN = 1 << 12
  NSTATE = 13
  PHYSICS = QPOS | QVEL | ACT
  FULLPHYSICS = TIME | PHYSICS | PLUGIN
  USER = CTRL | QFRC_APPLIED | XFRC_APPLIED | EQ_ACTIVE | MOCAP_POS | MOCAP_QUAT | USERDATA
  INTEGRATION = FULLPHYSICS | USER | WARMSTART


@dataclasses.dataclass
class Option:
  """Physics options (types.py:706-772).  Batched fields are (nb,) tensors."""

  timestep: Any = None
  tolerance: Any = None
  ls_tolerance: Any = None
  ccd_tolerance: Any = None
  density: Any = None
  viscosity: Any = None
  gravity: Any = None
  wind: Any = None
  magnetic: Any = None
  impratio_invsqrt: Any = None
  integrator: int = 0
  cone: int = 0
  solver: int = 2
  jacobian: int = 2
  iterations: int = 100
  ls_iterations: int = 50
  ccd_iterations: int = 35
  disableflags: int = 0
  enableflags: int = 0
  # warp-only fields (io.py:187-199)
  ls_parallel: bool = False
  ls_parallel_min_step: float = 1e-6
  broadphase: int = BroadphaseType.NXN
  broadphase_filter: int = BroadphaseFilter.PLANE | BroadphaseFilter.SPHERE | BroadphaseFilter.OBB
  graph_conditional: bool = True
  run_collision_detection: bool = True
  contact_sensor_maxmatch: int = 64


@dataclasses.dataclass
class Statistic:
  meaninertia: Any = None


@dataclasses.dataclass
class Callback:
  """User callbacks (types.py:810-830); the fused HIP path runs when all are None."""

  control: Optional[Callable] = None
  passive: Optional[Callable] = None
  act_dyn: Optional[Callable] = None
  act_gain: Optional[Callable] = None
  act_bias: Optional[Callable] = None
  contactfilter: Optional[Callable] = None


class _Container:
  """Attribute bag with a stable field order; used for Model / Data / Contact / Constraint."""

  def __init__(self, **kw):
    self.__dict__.update(kw)

  def fields(self):
    return list(self.__dict__.keys())

  def __repr__(self):
    names = ", ".join(self.__dict__.keys())
    return f"{type(self).__name__}({names})"


class Model(_Container):
  """Device model.  Field names follow mujoco_warp `types.Model` (types.py:833-1603)."""


class Data(_Container):
  """Device data.  Field names follow mujoco_warp `types.Data` (types.py:1702-1896)."""


class Contact(_Container):
  """Global contact pool (types.py:1617-1655): arrays of length naconmax, filled [0, nacon)."""


class Constraint(_Container):
  """Per-world constraint rows (types.py:1658-1699): (nworld, njmax[_pad]) arrays."""
