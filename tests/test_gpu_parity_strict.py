"""GPU parity at the north-star bar: HIP path vs the fp64 oracle at rtol 1e-5.

Tolerances (measured margins in profiles/r02_parity_report.json, tools/parity_report.py):
  * P0 smooth stages (kinematics, com, crb / qM, qLD, transmission, velocity, passive, rne, actuation,
    qfrc_smooth): elementwise rtol 1e-5 with an absolute floor of 1e-6 * scale, scale = max |oracle|
    of the field in that world.  Measured worst normwise error 3.8e-7.
  * Quantities behind a solve with M (qacc_smooth, and qvel / qacc after a step): fp32 Cholesky on a
    matrix of condition ~1e3 cannot be elementwise 1e-5 on near-zero components, so the bar is
    normwise (max |err| <= 1e-5 * max |oracle| per world) plus the backward error
    |M qacc - qfrc_smooth| <= 1e-5 |qfrc_smooth| evaluated in fp64.
Also covered here: nonzero xfrc_applied / qfrc_applied, per-world (batched `*`) model fields at
nb = nworld, nworld in {1, 7} (C1 sizes), and the device ctrl_noise kernel against the oracle formula.
"""

import copy

import numpy as np
import pytest

from tests.common import gpu_from_state, humanoid_model, np_, oracle_from_state, random_states

pytestmark = pytest.mark.gpu

RTOL = 1e-5
FLOOR = 1e-6

SMOOTH = {
  "fwd_position": ("xpos", "xquat", "xmat", "xipos", "ximat", "xanchor", "xaxis", "geom_xpos", "geom_xmat", "subtree_com", "cinert",
                   "cdof", "crb", "cam_xpos", "cam_xmat", "light_xpos", "light_xdir", "actuator_length"),
  "fwd_velocity": ("actuator_velocity", "cvel", "cdof_dot", "qfrc_spring", "qfrc_damper", "qfrc_passive", "qfrc_bias"),
  "fwd_actuation": ("actuator_force", "qfrc_actuator"),
  "fwd_acceleration": ("qfrc_smooth",),
}


def strict_close(name, got, want, rtol=RTOL, floor=FLOOR):
  """Elementwise |got - want| <= rtol |want| + floor * scale, scale = max |want| per world (row)."""
  got = np.asarray(got, np.float64).reshape(len(want), -1)
  want = np.asarray(want, np.float64).reshape(len(want), -1)
  scale = np.abs(want).max(axis=1, keepdims=True)
  err = np.abs(got - want)
  bad = err > rtol * np.abs(want) + floor * scale
  if bad.any():
    i = np.unravel_index(np.argmax(err / (rtol * np.abs(want) + floor * scale + 1e-300)), err.shape)
    raise AssertionError(f"{name}: {bad.sum()}/{bad.size} outside rtol {rtol} (+{floor}*scale); worst {i}: {got[i]} vs {want[i]}")


def normwise_close(name, got, want, tol=RTOL):
  got = np.asarray(got, np.float64).reshape(len(want), -1)
  want = np.asarray(want, np.float64).reshape(len(want), -1)
  e = np.abs(got - want).max(axis=1) / (np.abs(want).max(axis=1) + 1e-300)
  assert e.max() <= tol, f"{name}: normwise error {e.max():.3e} > {tol} (world {int(e.argmax())})"


def backward_close(name, qacc, od, nv, tol=RTOL):
  M = od.qM.reshape(-1, nv, nv)
  r = np.einsum("wij,wj->wi", M, qacc) - od.qfrc_smooth
  e = np.abs(r).max(axis=1) / (np.abs(od.qfrc_smooth).max(axis=1) + 1e-300)
  assert e.max() <= tol, f"{name}: backward error {e.max():.3e} > {tol}"


def _stages(mjw, m, d, od, check):
  import torch

  for st, fields in SMOOTH.items():
    getattr(mjw, st)(m, d)
    getattr(od, st)()
    torch.cuda.synchronize()
    for f in fields:
      check(f, np_(getattr(d, f)).reshape(d.nworld, -1), getattr(od, f))


@pytest.mark.parametrize("nworld", [1, 7, 32])
def test_smooth_stages_strict(nworld):
  """P0: every smooth-stage output at rtol 1e-5 (nworld 1 = C1's size, 7 = not a multiple of anything)."""
  import mujoco_warp_amd as mjw

  mjm = humanoid_model("CG")
  qpos, qvel, ctrl = random_states(mjm, nworld, seed=20 + nworld)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl)
  _stages(mjw, m, d, od, strict_close)
  nv = mjm.nv
  strict_close("qM", np_(d.qM)[:, :nv, :nv], od.qM)
  strict_close("qLD", np_(d.qLD), od.qLD)
  normwise_close("qacc_smooth", np_(d.qacc_smooth), od.qacc_smooth)
  backward_close("qacc_smooth", np_(d.qacc_smooth), od, nv)


def _no_efc_state(mjm, nworld, seed):
  k = mjm.key_names.index("no_efc")
  rng = np.random.default_rng(seed)
  qpos = np.tile(mjm.key_qpos[k], (nworld, 1))
  qvel = rng.normal(0, 0.2, (nworld, mjm.nv))
  ctrl = rng.uniform(-1, 1, (nworld, mjm.nu))
  return qpos, qvel, ctrl


@pytest.mark.parametrize("nworld", [1, 7])
def test_step_no_efc_strict(nworld):
  """P3: one full step from the contact-free key `no_efc` (humanoid.xml:245-250): nefc = 0 and
  qpos / qvel / qacc at 1e-5 (normwise per world; qpos elementwise)."""
  import torch

  import mujoco_warp_amd as mjw

  mjm = humanoid_model("CG")
  qpos, qvel, ctrl = _no_efc_state(mjm, nworld, seed=30)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl)
  mjw.step(m, d)
  od.step()
  torch.cuda.synchronize()
  assert int(np_(d.nefc).max()) == 0 and int(od.nefc.max()) == 0
  strict_close("qpos", np_(d.qpos), od.qpos)
  normwise_close("qvel", np_(d.qvel), od.qvel)
  normwise_close("qacc", np_(d.qacc), od.qacc)
  strict_close("time", np_(d.time).reshape(-1, 1), od.time)


def test_applied_forces_strict():
  """Nonzero xfrc_applied (xfrc_accumulate / apply_ft, support.py:174-237) and qfrc_applied enter
  qfrc_smooth and qacc_smooth exactly as in the oracle; then one step."""
  import torch

  import mujoco_warp_amd as mjw

  mjm = humanoid_model("CG")
  nworld = 16
  qpos, qvel, ctrl = random_states(mjm, nworld, seed=40)
  rng = np.random.default_rng(41)
  xfrc = rng.normal(0, 20.0, (nworld, mjm.nbody, 6))
  xfrc[:, 0] = 0.0  # the world body takes no applied force
  qfrc = rng.normal(0, 5.0, (nworld, mjm.nv))
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl)
  d.xfrc_applied[:] = torch.as_tensor(xfrc, dtype=torch.float32, device="cuda").reshape(d.xfrc_applied.shape)
  d.qfrc_applied[:] = torch.as_tensor(qfrc, dtype=torch.float32, device="cuda")
  od.xfrc_applied[:] = xfrc.reshape(nworld, -1)
  od.qfrc_applied[:] = qfrc
  _stages(mjw, m, d, od, strict_close)
  normwise_close("qacc_smooth", np_(d.qacc_smooth), od.qacc_smooth)
  backward_close("qacc_smooth", np_(d.qacc_smooth), od, mjm.nv)
  # the applied forces actually changed the result
  m0, d0 = gpu_from_state(mjm, qpos, qvel, ctrl)
  mjw.fwd_position(m0, d0)
  mjw.fwd_velocity(m0, d0)
  mjw.fwd_actuation(m0, d0)
  mjw.fwd_acceleration(m0, d0)
  torch.cuda.synchronize()
  assert np.abs(np_(d0.qfrc_smooth) - np_(d.qfrc_smooth)).max() > 1.0


def _per_world_models(mjm, nworld, rng):
  """nworld host models differing in gravity, timestep and body masses (the batched `*` fields)."""
  models = []
  for w in range(nworld):
    mw = copy.deepcopy(mjm)
    mw.opt.gravity = np.array([rng.normal(0, 0.5), rng.normal(0, 0.5), -9.81 * rng.uniform(0.5, 1.5)])
    mw.opt.timestep = float(mjm.opt.timestep * rng.uniform(0.5, 1.0))
    mw.body_mass = np.asarray(mjm.body_mass, np.float64) * np.concatenate([[1.0], rng.uniform(0.7, 1.3, mjm.nbody - 1)])
    models.append(mw)
  return models


def test_batched_model_fields():
  """Model fields with leading dim nb = nworld (reference io.py:59-63, read at worldid % nb): per-world
  opt.gravity, opt.timestep and body_mass.  Each world is checked against an oracle model built from
  that world's values: every smooth-stage output at the strict bar (this is where the batched fields
  enter), then the constraint solve at the solver bar (qacc normwise 5e-3, solver_test.py:32 -- the
  fp32 CG iterate, not the batching, sets that error; tools' batched probe measured smooth errors
  <= 2e-7 and solve errors 1e-4..1e-3 identical to unbatched runs), then one step (time exact)."""
  import torch

  import mujoco_warp_amd as mjw

  mjm = humanoid_model("CG")
  nworld = 8
  rng = np.random.default_rng(50)
  models = _per_world_models(mjm, nworld, rng)
  qpos, qvel, ctrl = random_states(mjm, nworld, seed=51)

  def batched(m):
    dev = m.opt.gravity.device
    m.opt.gravity = torch.as_tensor(np.stack([mw.opt.gravity for mw in models]), dtype=torch.float32, device=dev)
    m.opt.timestep = torch.as_tensor([mw.opt.timestep for mw in models], dtype=torch.float32, device=dev)
    m.body_mass = torch.as_tensor(np.stack([mw.body_mass for mw in models]), dtype=torch.float32, device=dev)

  m, d = gpu_from_state(mjm, qpos, qvel, ctrl)
  batched(m)
  for st in SMOOTH:
    getattr(mjw, st)(m, d)
  mjw.solve(m, d)
  m2, d2 = gpu_from_state(mjm, qpos, qvel, ctrl)
  batched(m2)
  mjw.step(m2, d2)
  torch.cuda.synchronize()
  nv = mjm.nv
  for w, mw in enumerate(models):
    om, od = oracle_from_state(mw, qpos[w : w + 1], qvel[w : w + 1], ctrl[w : w + 1])
    for st in SMOOTH:
      getattr(od, st)()
    for f in ("cinert", "crb", "qfrc_bias", "qfrc_passive", "qfrc_smooth"):
      strict_close(f"{f}[w{w}]", np_(getattr(d, f)).reshape(nworld, -1)[w : w + 1], getattr(od, f))
    strict_close(f"qM[w{w}]", np_(d.qM)[w : w + 1, :nv, :nv], od.qM)
    normwise_close(f"qacc_smooth[w{w}]", np_(d.qacc_smooth)[w : w + 1], od.qacc_smooth)
    od.solve()
    normwise_close(f"qacc[w{w}]", np_(d.qacc)[w : w + 1], od.qacc, tol=5e-3)
    om2, od2 = oracle_from_state(mw, qpos[w : w + 1], qvel[w : w + 1], ctrl[w : w + 1])
    od2.step()
    strict_close(f"time[w{w}]", np_(d2.time)[w : w + 1].reshape(1, 1), od2.time)
    normwise_close(f"qpos[w{w}]", np_(d2.qpos)[w : w + 1], od2.qpos, tol=1e-4)
  t = np_(d2.time)
  assert len(np.unique(t)) == nworld  # per-world timesteps really took effect


@pytest.mark.parametrize("world_offset", [0, 8192 * 3 + 5])
def test_ctrl_noise_device_vs_oracle(world_offset):
  """The device ctrl_noise kernel (mjw_step.hip) against the oracle's restatement of
  benchmark.py:41-83 (OU + Halton with global world ids) over 5 steps, with and without a center."""
  import torch

  import mujoco_warp_amd as mjw

  mjm = humanoid_model("CG")
  nworld = 64
  qpos, qvel, _ = random_states(mjm, nworld, seed=60)
  ctrl0 = np.zeros((nworld, mjm.nu))
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl0)
  d.world_offset = world_offset
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl0)
  center = np.asarray(mjm.key_ctrl[0], np.float64) + 0.1
  ct = torch.as_tensor(center, dtype=torch.float32, device="cuda")
  for i in range(5):
    c = None if i % 2 == 0 else ct
    mjw.ctrl_noise(m, d, i, center=c)
    od.ctrl_noise(i, center=None if c is None else center, world_offset=world_offset)
    torch.cuda.synchronize()
    got, want = np_(d.ctrl), od.ctrl
    assert np.abs(got - want).max() <= 1e-6 * max(1.0, np.abs(want).max()), f"step {i}: {np.abs(got - want).max()}"
  assert np.abs(np_(d.ctrl)).max() > 0


def test_constraint_rows_strict():
  """P1: contacts and constraint rows of 32 contact-rich worlds.  Counts, row order and types are
  identical; J and efc_vel at the strict bar; contact dist and efc_pos to 1e-6 m absolute (a distance
  is a difference of ~1 m coordinates, so fp32 round-off is ~1e-7 m whatever its size); efc_D and
  efc_aref at rtol 3e-4, which is that 1e-7 m position round-off carried through the impedance
  curve (d imp / d pos ~ 1 / solimp width, width 0.001-0.01 m in humanoid.xml)."""
  import torch

  import mujoco_warp_amd as mjw

  mjm = humanoid_model("CG")
  nworld = 32
  nv = mjm.nv
  qpos, qvel, ctrl = random_states(mjm, nworld, seed=70)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl)
  mjw.fwd_position(m, d)
  od.fwd_position()
  torch.cuda.synchronize()
  nacon = int(d.nacon[0])
  gw = np_(d.contact.worldid[:nacon]).astype(int)
  total = 0
  for w in range(nworld):
    n = int(d.nefc[w])
    assert n == int(od.nefc[w, 0]) and int(d.nl[w]) == int(od.nl[w, 0]) and int(d.nf[w]) == int(od.nf[w, 0])
    assert np.array_equal(d.efc.type[w, :n].cpu().numpy(), od.efc_type[w, :n])
    sel = np.nonzero(gw == w)[0]
    assert len(sel) == int(od.ncon[w, 0])
    if len(sel):
      assert np.abs(np.sort(np_(d.contact.dist[:nacon])[sel]) - np.sort(od.con_dist[w, : len(sel)])).max() <= 1e-6
    if n == 0:
      continue
    total += n
    strict_close(f"efc.J[w{w}]", np_(d.efc.J[w, :n, :nv]).reshape(1, -1), od.efc_J[w].reshape(od.njmax, nv)[:n].reshape(1, -1))
    strict_close(f"efc.vel[w{w}]", np_(d.efc.vel[w, :n])[None], od.efc_vel[w, :n][None])
    assert np.array_equal(np_(d.efc.margin[w, :n]), od.efc_margin[w, :n].astype(np.float32).astype(np.float64))
    assert np.abs(np_(d.efc.pos[w, :n]) - od.efc_pos[w, :n]).max() <= 1e-6
    for f in ("D", "aref"):
      strict_close(f"efc.{f}[w{w}]", np_(getattr(d.efc, f)[w, :n])[None], getattr(od, "efc_" + f)[w, :n][None], rtol=3e-4)
  assert total > 10 * nworld


@pytest.mark.parametrize("solver", ["CG", "NEWTON"])
def test_step_with_contacts_nworld1(solver):
  """C1 (humanoid, nworld = 1) through a contact step: the rows agree (count, type, order), the solve
  from the same smooth state reaches the oracle's optimum (fp64 primal cost of the oracle's rows:
  relative excess <= 1e-5, the reference's bar being 2.5 %, solver_test.py:308-322) with qacc
  normwise 5e-3 (solver_test.py:32), and one full step gives qpos normwise 1e-5 and qvel 5e-3."""
  import torch

  import mujoco_warp_amd as mjw
  from tests.parity_models import efc_cost

  mjm = humanoid_model(solver)
  nv = mjm.nv
  for seed in range(80, 120):  # the first state whose feet touch the floor
    qpos, qvel, ctrl = random_states(mjm, 1, seed=seed)
    om, od = oracle_from_state(mjm, qpos, qvel, ctrl)
    od.fwd_position()
    if int(od.nefc[0, 0]) >= 8:
      break
  n = int(od.nefc[0, 0])
  assert n >= 8
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl)
  for st in SMOOTH:
    getattr(mjw, st)(m, d)
    getattr(od, st)()
  mjw.solve(m, d)
  od.solve()
  torch.cuda.synchronize()
  assert int(d.nefc[0]) == n
  assert np.array_equal(d.efc.type[0, :n].cpu().numpy(), od.efc_type[0, :n])
  J = od.efc_J[0].reshape(od.njmax, nv)[:n]
  M = od.qM[0].reshape(nv, nv)
  args = (J, od.efc_D[0, :n], od.efc_aref[0, :n], od.efc_type[0, :n], M, od.qacc_smooth[0])
  c_or = efc_cost(*args, od.qacc[0], fl=od.efc_frictionloss[0, :n])
  c_gpu = efc_cost(*args, np_(d.qacc[0]), fl=od.efc_frictionloss[0, :n])
  assert (c_gpu - c_or) / abs(c_or) <= 1e-5, (c_gpu, c_or)
  normwise_close("qacc", np_(d.qacc), od.qacc, tol=5e-3)
  m2, d2 = gpu_from_state(mjm, qpos, qvel, ctrl)
  om2, od2 = oracle_from_state(mjm, qpos, qvel, ctrl)
  mjw.step(m2, d2)
  od2.step()
  torch.cuda.synchronize()
  normwise_close("qpos", np_(d2.qpos), od2.qpos)
  normwise_close("qvel", np_(d2.qvel), od2.qvel, tol=5e-3)
