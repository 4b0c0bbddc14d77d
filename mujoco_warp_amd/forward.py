"""Pipeline entry points (mirror mujoco_warp/_src/forward.py).

`step(m, d)` (forward.py:1003-1018) runs the whole forward pass and the Euler
integrator on the current torch stream as two world-per-wavefront HIP kernels:
the forward kernel (kinematics ... qfrc_smooth, collision and constraint rows)
and, for models with nv <= 32 and njmax <= 64, the register-resident dense
factor / solve / integrate kernel (otherwise one generic fused kernel).  The
stage functions (`fwd_position`, `fwd_velocity`, ...) launch the
same device code restricted to one stage group; they exist for parity testing
and for models that install Python callbacks (types.Callback), which are
invoked between stage launches exactly where the reference calls them.
"""

from __future__ import annotations

import torch

from . import _lib
from .io import cdata, cmodel
from .types import Data, DisableBit, EnableBit, IntegratorType, Model


def _stream(d: Data):
  if d.device.type != "cuda":
    raise RuntimeError("mujoco_warp_amd runs on the ROCm device only (no CPU fallback): pass device='cuda'")
  return torch.cuda.current_stream(d.device).cuda_stream


def _call(fn: str, m: Model, d: Data):
  L = _lib.lib()
  cm, cd = cmodel(m), cdata(d)
  _lib.check(getattr(L, fn)(cm, cd, _stream(d)), fn)


def step_timed(m: Model, d: Data, ev_begin, ev_mid, ev_end):
  """`step` that records torch.cuda.Event objects around its kernels (bench.py).

  The events must already exist (torch creates them on their first `record()`)."""
  for e in (ev_begin, ev_mid, ev_end):
    if not e.cuda_event:
      raise ValueError("step_timed: record each event once before passing it")
  L = _lib.lib()
  rc = L.mjw_step_events(cmodel(m), cdata(d), _stream(d), ev_begin.cuda_event, ev_mid.cuda_event, ev_end.cuda_event)
  _lib.check(rc, "mjw_step_events")


class StepTracer:
  """Times every kernel launch of `step` with HIP events on the stream the kernels run on
  (mjw_step_trace).  `step(m, d)` runs one traced step; `durations()` then gives, per traced step, the
  list of (kernel name, ms) in launch order (call after the work has finished)."""

  def __init__(self, max_launch: int = 32):
    import ctypes

    self._ct = ctypes
    self.max_launch = max_launch
    self.records = []  # (events, ids, n) per traced step

  def step(self, m: Model, d: Data):
    ct = self._ct
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(self.max_launch + 1)]
    for e in evs:  # torch creates the HIP event on its first record
      e.record()
    arr = (ct.c_void_p * len(evs))(*[e.cuda_event for e in evs])
    ids = (ct.c_int * self.max_launch)()
    n = ct.c_int(0)
    _lib.check(_lib.lib().mjw_step_trace(cmodel(m), cdata(d), _stream(d), arr, len(evs), ids, ct.byref(n)), "mjw_step_trace")
    self.records.append((evs, [ids[i] for i in range(n.value)], n.value))

  def durations(self):
    L = _lib.lib()
    out = []
    for evs, ids, n in self.records:
      out.append([(L.mjw_kernel_name(ids[i]).decode(), evs[i].elapsed_time(evs[i + 1])) for i in range(n)])
    return out


# callbacks whose reference call sites fall inside one fused launch of this path (none left: contactfilter,
# between the narrowphase and make_constraint, runs after the position stage, which then rebuilds the
# constraint rows from the contact pool it edited -- mjw_contact_rows)
_UNSUPPORTED_CALLBACKS: dict = {}
_STAGED_CALLBACKS = ("control", "passive", "act_dyn", "act_gain", "act_bias", "contactfilter")


def _has_callbacks(m: Model) -> bool:
  cb = m.callback
  for f, where in _UNSUPPORTED_CALLBACKS.items():
    if getattr(cb, f) is not None:
      raise NotImplementedError(f"callback.{f} (called at reference {where}) is not supported: the stage it hooks into is one fused HIP launch")
  return any(getattr(cb, f) is not None for f in _STAGED_CALLBACKS)


def fwd_position(m: Model, d: Data):
  """Position-dependent computations (forward.py:513-537).  A contactfilter callback runs after the
  narrowphase wrote d.contact (collision_driver.py:788-789); the constraint rows (make_constraint, which
  the reference runs after it) are then rebuilt from the contacts as the callback left them
  (mjw_contact_rows: contacts whose `type` lost the CONSTRAINT bit get no rows)."""
  _has_callbacks(m)
  _call("mjw_fwd_position", m, d)
  if m.callback.contactfilter is not None:
    if d.naconmax > 0 and not (m.opt.disableflags & (DisableBit.CONSTRAINT | DisableBit.CONTACT)):
      m.callback.contactfilter(m, d)
      _call("mjw_contact_rows", m, d)


def fwd_velocity(m: Model, d: Data):
  """Velocity-dependent computations (forward.py:592-613)."""
  _call("mjw_fwd_velocity", m, d)
  if m.callback.passive is not None:
    m.callback.passive(m, d)


def fwd_actuation(m: Model, d: Data):
  """Actuation-dependent computations (forward.py:836-927).  With act_dyn / act_gain / act_bias
  callbacks: actuator force and act_dot first, then the callbacks in the reference's order
  (forward.py:876-881), then the moment map qfrc_actuator = moment' actuator_force from the forces the
  callbacks left (mjw_actuator_map)."""
  _has_callbacks(m)
  _call("mjw_fwd_actuation", m, d)
  cb = m.callback
  act_cbs = [f for f in (cb.act_dyn, cb.act_gain, cb.act_bias) if f is not None]
  if act_cbs and m.nu and not (m.opt.disableflags & DisableBit.ACTUATION):
    for f in act_cbs:
      f(m, d)
    _call("mjw_actuator_map", m, d)


def fwd_acceleration(m: Model, d: Data, factorize: bool = True):
  """qfrc_smooth and qacc_smooth (forward.py:949-969); always factorizes qM."""
  _call("mjw_fwd_acceleration", m, d)


def solve(m: Model, d: Data):
  """Constraint solver (solver.py:3296-3343)."""
  _call("mjw_solve", m, d)


def euler(m: Model, d: Data):
  """Euler integrator, semi-implicit in velocity (forward.py:326-354)."""
  _call("mjw_euler", m, d)


def _sensor(m: Model, d: Data, stages: int):
  L = _lib.lib()
  _lib.check(L.mjw_sensor(cmodel(m), cdata(d), int(stages), _stream(d)), "mjw_sensor")


def sensor_pos(m: Model, d: Data):
  """Position-dependent sensors (sensor.py:761); valid after fwd_position."""
  _sensor(m, d, 1)


def sensor_vel(m: Model, d: Data):
  """Velocity-dependent sensors (sensor.py:1377); valid after fwd_velocity."""
  _sensor(m, d, 2)


def sensor_acc(m: Model, d: Data):
  """Acceleration-dependent sensors with rne_postconstraint (sensor.py:2447); valid after solve."""
  _sensor(m, d, 4)


def implicit(m: Model, d: Data):
  """Implicit-in-velocity integration (forward.py:494-510); the integrator kernel dispatches on
  opt.integrator, so this is the same launch as `euler` for implicitfast models."""
  _call("mjw_euler", m, d)


def _rk4_op(m: Model, d: Data, op: int, scale: float):
  L = _lib.lib()
  _lib.check(L.mjw_rk4_op(cmodel(m), cdata(d), int(op), float(scale), _stream(d)), "mjw_rk4_op")


def rungekutta4(m: Model, d: Data):
  """Runge-Kutta explicit order 4 integrator (forward.py:457-491); call after `forward`.

  Without Python callbacks the three inner forward passes and the bookkeeping run inside the
  library (mjw_rungekutta4); with callbacks the inner passes go through `forward` here so the
  callbacks see every stage, and the bookkeeping launches the same device ops one by one."""
  if not (_has_callbacks(m) or _energy(m)):
    _call("mjw_rungekutta4", m, d)
    return
  A = (0.5, 0.5, 1.0)
  B = (1.0 / 6.0, 1.0 / 3.0, 1.0 / 3.0, 1.0 / 6.0)
  _rk4_op(m, d, 0, B[0])
  for i in range(3):
    _rk4_op(m, d, 1, A[i])
    forward(m, d)
    _rk4_op(m, d, 2, B[i + 1])
  _rk4_op(m, d, 3, 0.0)


def _integrate(m: Model, d: Data):
  if m.opt.integrator == IntegratorType.RK4:
    rungekutta4(m, d)
  else:
    euler(m, d)


def step1(m: Model, d: Data):
  """First half of `step` (forward.py:1022-1047): position and velocity stages with their sensors, the
  potential / kinetic energy after each when ENERGY is enabled (else d.energy is cleared), then the
  control callback."""
  from .stages import energy_pos, energy_vel

  fwd_position(m, d)
  sensor_pos(m, d)
  if _energy(m):
    energy_pos(m, d)
  else:
    d.energy.zero_()
  fwd_velocity(m, d)
  sensor_vel(m, d)
  if _energy(m):
    energy_vel(m, d)
  if not (m.opt.disableflags & DisableBit.ACTUATION) and m.callback.control is not None:
    m.callback.control(m, d)


def step2(m: Model, d: Data):
  """Second half of `step` after the user has set its inputs (forward.py:1050-1064): actuation,
  acceleration, solver, acceleration sensors, integration -- implicitfast for implicitfast models, Euler
  otherwise (the reference's step2 integrates RK4 models with Euler, forward.py:1063)."""
  fwd_actuation(m, d)
  fwd_acceleration(m, d)
  solve(m, d)
  sensor_acc(m, d)
  euler(m, d)  # mjw_euler dispatches on opt.integrator: implicitfast, else Euler (RK4 included)


def _energy(m: Model) -> bool:
  """opt.enableflags ENERGY: potential / kinetic energy into d.energy (forward.py:975-991), computed on the
  staged path right after the position and velocity stages, as the reference does."""
  return bool(m.opt.enableflags & EnableBit.ENERGY)


def _forward_staged(m: Model, d: Data):
  from .stages import energy_pos, energy_vel

  fwd_position(m, d)
  if _energy(m):
    energy_pos(m, d)
  fwd_velocity(m, d)
  if _energy(m):
    energy_vel(m, d)
  if not (m.opt.disableflags & DisableBit.ACTUATION) and m.callback.control is not None:
    m.callback.control(m, d)
  fwd_actuation(m, d)
  fwd_acceleration(m, d)
  solve(m, d)
  _sensor(m, d, 7)


def forward(m: Model, d: Data):
  """Forward dynamics (forward.py:972-1000)."""
  if _has_callbacks(m) or _energy(m):
    _forward_staged(m, d)
  else:
    _call("mjw_forward", m, d)


def step(m: Model, d: Data):
  """Advance simulation (forward.py:1003-1018)."""
  if _has_callbacks(m) or _energy(m):
    _forward_staged(m, d)
    _integrate(m, d)
  else:
    _call("mjw_step", m, d)


def ctrl_noise(m: Model, d: Data, step_index: int, center: torch.Tensor | None = None, std: float = 0.01, rate: float = 0.1):
  """Per-step OU + Halton control noise of the reference benchmark (_src/benchmark.py:41-83)."""
  L = _lib.lib()
  ptr = None if center is None or center.numel() == 0 else center.data_ptr()
  _lib.check(L.mjw_ctrl_noise(cmodel(m), cdata(d), ptr, int(step_index), float(std), float(rate), _stream(d)), "mjw_ctrl_noise")
