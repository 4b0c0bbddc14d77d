"""RK4 integrator (forward.py:357-491) and activation dynamics (forward.py:616-697 act_dot / actearly,
support.py:38-64 next_act) -- SURVEY.md §8(a) integrator rows.

Oracle pinning (CPU): RK4's global error is 4th order in the timestep on a spring-mass system with a
closed-form solution; FILTEREXACT integrates a constant-input first-order filter exactly; an
integrator actuator ramps linearly and clamps to actrange; actearly makes the force see the next
step's activation.  `-m gpu`: the device RK4 / activation path against the fp64 oracle on a model that
has every supported activation type, and on humanoid; the callback path (Python-driven RK4 stages)
against the fused one.
"""

import numpy as np
import pytest

from tests.common import assert_close, gpu_from_state, humanoid_model, np_, oracle_from_state

ACT_XML = """<mujoco><option timestep="0.005" integrator="{integrator}"/><worldbody>
<geom type="plane" size="5 5 .1"/>
<body pos="0 0 1"><joint name="h1" type="hinge" axis="0 1 0" damping="0.1"/>
  <geom type="capsule" fromto="0 0 0 .3 0 0" size=".04"/>
  <body pos=".3 0 0"><joint name="h2" type="hinge" axis="0 1 0"/><geom type="capsule" fromto="0 0 0 .3 0 0" size=".04"/>
    <body pos=".3 0 0"><joint name="s3" type="slide" axis="1 0 0" stiffness="20"/><geom type="sphere" size=".05"/></body>
  </body>
</body>
<body pos="1 0 .3"><freejoint/><geom type="sphere" size=".1"/></body>
<body pos="-1 0 .5"><joint type="ball" name="b"/><geom type="capsule" fromto="0 0 0 0 .2 -.2" size=".03"/></body>
</worldbody><actuator>
<intvelocity joint="h1" kp="30" actrange="-1 1"/>
<position joint="h2" kp="20" kv="1" timeconst="0.05"/>
<general joint="s3" dyntype="filter" dynprm="0.03" gainprm="5"/>
<general joint="h2" dyntype="integrator" actearly="true" actlimited="true" actrange="-.5 .5" gainprm="2"/>
<motor joint="h1" gear="2"/>
</actuator></mujoco>"""

SPRING_XML = """<mujoco><option timestep="{h}" integrator="{integrator}" gravity="0 0 0"/><worldbody>
<body><joint name="x" type="slide" axis="1 0 0" stiffness="{k}"/><inertial pos="0 0 0" mass="{mass}" diaginertia=".1 .1 .1"/></body>
</worldbody></mujoco>"""


def _load(xml):
  from mujoco_warp_amd import mjcf

  return mjcf.load_model_from_string(xml)


def _oracle(mjm, nworld=1, qpos=None, qvel=None, ctrl=None):
  qpos = np.tile(mjm.qpos0, (nworld, 1)) if qpos is None else qpos
  qvel = np.zeros((nworld, mjm.nv)) if qvel is None else qvel
  ctrl = np.zeros((nworld, mjm.nu)) if ctrl is None else ctrl
  return oracle_from_state(mjm, qpos, qvel, ctrl)


def _act_states(mjm, nworld, seed):
  rng = np.random.default_rng(seed)
  qpos = np.tile(mjm.qpos0, (nworld, 1))
  qpos[:, :3] += rng.normal(0, 0.3, (nworld, 3))
  q = np.tile([1.0, 0, 0, 0], (nworld, 1)) + rng.normal(0, 0.2, (nworld, 4))
  qpos[:, -4:] = q / np.linalg.norm(q, axis=1, keepdims=True)  # ball joint
  qvel = rng.normal(0, 0.5, (nworld, mjm.nv))
  ctrl = rng.uniform(-1, 1, (nworld, mjm.nu))
  act = rng.uniform(-0.4, 0.4, (nworld, mjm.na))
  return qpos, qvel, ctrl, act


# ---- CPU: oracle pinning -----------------------------------------------------------------------
def test_oracle_rk4_is_fourth_order():
  k, mass, x0, T = 40.0, 2.0, 0.1, 1.0
  w = np.sqrt(k / mass)
  errs = {}
  for integ in ("RK4", "Euler"):
    for h in (0.02, 0.01):
      mjm = _load(SPRING_XML.format(h=h, integrator=integ, k=k, mass=mass))
      om, od = _oracle(mjm, qpos=np.array([[x0]]))
      for _ in range(int(round(T / h))):
        od.step()
      errs[integ, h] = abs(od.qpos[0, 0] - x0 * np.cos(w * T))
      assert abs(od.time[0, 0] - T) < 1e-12
  assert errs["RK4", 0.01] < 1e-6
  ratio = errs["RK4", 0.02] / errs["RK4", 0.01]
  assert 12 < ratio < 20, ratio  # 2^4
  assert errs["Euler", 0.01] > 100 * errs["RK4", 0.01]


def test_oracle_activation_dynamics_closed_forms():
  mjm = _load(ACT_XML.format(integrator="Euler"))
  mjm.opt.gravity[:] = 0
  mjm.opt.disableflags |= 1  # no constraints
  assert mjm.na == 4 and list(mjm.actuator_dyntype) == [1, 3, 2, 1, 0]
  h, n = mjm.opt.timestep, 120
  u = np.array([[0.3, 0.8, -0.6, 0.9, 0.0]])
  om, od = _oracle(mjm, ctrl=u)
  for _ in range(n):
    od.step()
  tau_fe, tau_f = mjm.actuator_dynprm[1, 0], mjm.actuator_dynprm[2, 0]
  want = [
    np.clip(0.3 * n * h, -1, 1),  # integrator, actrange [-1, 1]
    0.8 * (1 - np.exp(-n * h / tau_fe)),  # filterexact: exact for constant input
    -0.6 * (1 - (1 - h / tau_f) ** n),  # filter: explicit Euler recursion
    min(0.9 * n * h, 0.5),  # integrator clamped at actrange[1] (0.54 -> 0.5)
  ]
  np.testing.assert_allclose(od.act[0], want, rtol=1e-12, atol=1e-12)
  assert od.act_dot[0, 0] == 0.3 and od.act_dot[0, 3] == 0.9  # integrators: act_dot = ctrl


def test_oracle_actearly_force_sees_next_activation():
  mjm = _load(ACT_XML.format(integrator="Euler"))
  h = mjm.opt.timestep
  act = np.array([[0.1, 0.2, 0.3, 0.48]])
  u = np.array([[0.5, -0.5, 0.25, 0.9, 0.0]])
  om, od = _oracle(mjm, ctrl=u)
  od.act[:] = act
  od.forward()
  # actuator 3: integrator, actearly, actrange [-.5, .5], gain 2 -> force = 2 * clamp(.48 + .9 h)
  assert abs(od.actuator_force[0, 3] - 2 * min(0.48 + 0.9 * h, 0.5)) < 1e-12
  # actuator 2: filter (not early) -> force = 5 * act
  assert abs(od.actuator_force[0, 2] - 5 * 0.3) < 1e-12
  np.testing.assert_allclose(od.act_dot[0], [0.5, (-0.5 - 0.2) / 0.05, (0.25 - 0.3) / 0.03, 0.9], rtol=1e-12)


def test_oracle_rk4_free_and_ball_quaternions_stay_unit():
  mjm = _load(ACT_XML.format(integrator="RK4"))
  qpos, qvel, ctrl, act = _act_states(mjm, 4, seed=3)
  om, od = _oracle(mjm, 4, qpos, qvel * 4, ctrl)
  od.act[:] = act
  for _ in range(50):
    od.step()
  for adr in (mjm.jnt_qposadr[3] + 3, mjm.jnt_qposadr[4]):
    np.testing.assert_allclose(np.linalg.norm(od.qpos[:, adr : adr + 4], axis=1), 1.0, atol=1e-12)
  assert np.isfinite(od.qpos).all()


def test_put_model_accepts_rk4_rejects_muscle_without_lengthrange():
  """RK4 is accepted; a muscle activation on an actuator whose length range is unknown (no lengthrange
  attribute, unlimited joint) is refused rather than run with a degenerate range."""
  import mujoco_warp_amd as mjw

  mjm = _load(ACT_XML.format(integrator="RK4"))
  m = mjw.put_model(mjm, device="cpu")
  d = mjw.make_data(mjm, nworld=2, device="cpu", m=m)
  assert d.qpos_t0.shape == (2, mjm.nq) and d.act_dot_rk.shape == (2, mjm.na)
  xml = ACT_XML.format(integrator="Euler").replace('dyntype="filter" dynprm="0.03"', 'dyntype="muscle"')
  with pytest.raises(NotImplementedError, match="muscle"):
    mjw.put_model(_load(xml), device="cpu")


# ---- GPU: device vs oracle ---------------------------------------------------------------------
def _gpu_oracle_pair(mjm, nworld, seed, njmax=32, nconmax=8):
  import torch

  qpos, qvel, ctrl, act = _act_states(mjm, nworld, seed)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=njmax, nconmax=nconmax)
  d.act[:] = torch.as_tensor(act, dtype=torch.float32, device="cuda")
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=njmax, nconmax=nconmax)
  od.act[:] = act
  return m, d, od


@pytest.mark.gpu
@pytest.mark.parametrize("integrator", ["Euler", "RK4", "implicitfast"])
def test_gpu_activation_integrators_parity(integrator):
  import torch

  import mujoco_warp_amd as mjw

  mjm = _load(ACT_XML.format(integrator=integrator))
  m, d, od = _gpu_oracle_pair(mjm, 32, seed=11)
  for _ in range(20):
    mjw.step(m, d)
    od.step()
  torch.cuda.synchronize()
  assert_close("act", np_(d.act), od.act, rtol=1e-3, atol=1e-4)
  assert_close("act_dot", np_(d.act_dot), od.act_dot, rtol=2e-3, atol=2e-3)
  assert_close("qpos", np_(d.qpos), od.qpos, rtol=1e-3, atol=1e-3)
  assert_close("qvel", np_(d.qvel), od.qvel, rtol=5e-3, atol=5e-3)
  assert_close("time", np_(d.time), od.time[:, 0], rtol=1e-6, atol=0)


@pytest.mark.gpu
def test_gpu_rk4_humanoid_parity():
  import torch

  import mujoco_warp_amd as mjw
  from tests.common import random_states

  mjm = humanoid_model("NEWTON")
  mjm.opt.integrator = 1  # RK4
  qpos, qvel, ctrl = random_states(mjm, 32, seed=12)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=64, nconmax=24)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=64, nconmax=24)
  for _ in range(5):
    mjw.step(m, d)
    od.step()
  torch.cuda.synchronize()
  assert_close("qpos", np_(d.qpos), od.qpos, rtol=2e-3, atol=2e-3)
  assert_close("qvel", np_(d.qvel), od.qvel, rtol=2e-2, atol=2e-2)
  assert_close("qacc_warmstart", np_(d.qacc_warmstart), od.qacc_warmstart, rtol=5e-2, atol=5e-1)


@pytest.mark.gpu
def test_gpu_rk4_callback_path_matches_fused():
  import torch

  import mujoco_warp_amd as mjw

  mjm = _load(ACT_XML.format(integrator="RK4"))
  m, d, _ = _gpu_oracle_pair(mjm, 16, seed=13)
  m2, d2, _ = _gpu_oracle_pair(mjm, 16, seed=13)
  calls = []
  m2.callback.control = lambda mm, dd: calls.append(1)
  for _ in range(3):
    mjw.step(m, d)
    mjw.step(m2, d2)
  torch.cuda.synchronize()
  assert len(calls) == 3 * 4  # forward + three RK stages per step
  for name in ("qpos", "qvel", "act", "act_dot", "qacc_warmstart", "time"):
    np.testing.assert_array_equal(np_(getattr(d, name)), np_(getattr(d2, name)), err_msg=name)
