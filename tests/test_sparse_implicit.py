"""implicitfast on the sparse / flex path (csrc/mjw_sparse.hip euler_kernel): M - dt qDeriv assembled on
the sparse ancestor rows (forward.py:494-510, derivative.py:320-416), factored per tree.

A 3-link hinge chain with position actuators (kv enters qDeriv off the diagonal through the chain's
ancestor pattern) and dof damping, forced onto the sparse path with jacobian="sparse", against the
fp64 oracle and against the same model on the dense path; then aloha_cloth (flex towel, mesh arms,
position actuators) stepped with implicitfast against the oracle at the solver bar."""

import numpy as np
import pytest

from tests.common import gpu_from_state, np_, oracle_from_state

CHAIN = """<mujoco><option timestep="0.01" integrator="implicitfast" solver="CG" gravity="0 0 -9.81" jacobian="{jac}"/>
<worldbody>
  <body pos="0 0 1"><joint name="j0" type="hinge" axis="0 1 0" damping="0.3"/>
    <geom type="capsule" fromto="0 0 0 0 0 -0.4" size="0.04" contype="0" conaffinity="0"/>
    <body pos="0 0 -0.4"><joint name="j1" type="hinge" axis="0 1 0" damping="0.2"/>
      <geom type="capsule" fromto="0 0 0 0 0 -0.4" size="0.04" contype="0" conaffinity="0"/>
      <body pos="0 0 -0.4"><joint name="j2" type="hinge" axis="1 0 0" damping="0.1"/>
        <geom type="capsule" fromto="0 0 0 0 0 -0.3" size="0.03" contype="0" conaffinity="0"/>
      </body>
    </body>
  </body>
</worldbody>
<actuator>
  <position joint="j0" kp="40" kv="3"/>
  <position joint="j1" kp="30" kv="2"/>
  <position joint="j2" kp="20" kv="1"/>
</actuator></mujoco>"""


def _chain(jac):
  from mujoco_warp_amd import mjcf

  return mjcf.load_model_from_string(CHAIN.format(jac=jac))


def test_chain_compiles_sparse():
  import mujoco_warp_amd as mjw

  m = mjw.put_model(_chain("sparse"), device="cpu")
  assert m.is_sparse and int(m.opt.integrator) == 3


@pytest.mark.gpu
def test_gpu_sparse_implicitfast_matches_oracle_and_dense():
  import torch

  import mujoco_warp_amd as mjw

  nworld = 8
  rng = np.random.default_rng(3)
  ms = _chain("sparse")
  qpos = rng.normal(0, 0.3, (nworld, ms.nq))
  qvel = rng.normal(0, 2.0, (nworld, ms.nv))
  ctrl = rng.uniform(-0.5, 0.5, (nworld, ms.nu))
  m, d = gpu_from_state(ms, qpos, qvel, ctrl, njmax=8, nconmax=4)
  m2, d2 = gpu_from_state(_chain("dense"), qpos, qvel, ctrl, njmax=8, nconmax=4)
  om, od = oracle_from_state(ms, qpos, qvel, ctrl, njmax=8, nconmax=4)
  assert m.is_sparse and not m2.is_sparse
  for _ in range(3):
    mjw.step(m, d)
    mjw.step(m2, d2)
    od.step()
  torch.cuda.synchronize()
  from tests.test_gpu_parity_strict import normwise_close

  # no constraint rows: the step is the smooth dynamics and the implicit solve only
  normwise_close("qvel", np_(d.qvel), od.qvel)
  normwise_close("qpos", np_(d.qpos), od.qpos)
  normwise_close("qvel sparse vs dense", np_(d.qvel), np_(d2.qvel))
  # the implicit terms matter: the same steps with semi-implicit Euler land far outside the tolerance
  from mujoco_warp_amd import mjcf

  me = mjcf.load_model_from_string(CHAIN.format(jac="sparse").replace('integrator="implicitfast"', 'integrator="Euler"'))
  m3, d3 = gpu_from_state(me, qpos, qvel, ctrl, njmax=8, nconmax=4)
  for _ in range(3):
    mjw.step(m3, d3)
  torch.cuda.synchronize()
  e = np.abs(np_(d3.qvel) - od.qvel).max() / np.abs(od.qvel).max()
  assert e > 1e-3, e


@pytest.mark.gpu
def test_gpu_aloha_cloth_implicitfast_step():
  import torch

  import mujoco_warp_amd as mjw
  from tests.cloth_common import aloha_model, aloha_states
  from tests.test_gpu_parity_strict import normwise_close

  mjm = aloha_model()
  mjw.override_model(mjm, ["opt.integrator=implicitfast"])
  qpos, qvel, ctrl = aloha_states(mjm, 2, seed=5)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=16384, nconmax=4096)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=16384, nconmax=4096)
  assert m.is_sparse
  mjw.step(m, d)
  od.step()
  torch.cuda.synchronize()
  normwise_close("qpos", np_(d.qpos), od.qpos)
  normwise_close("qvel", np_(d.qvel), od.qvel, tol=5e-3)  # carries the CG solve (solver_test.py:32)


SENSED = CHAIN.replace('<geom type="capsule" fromto="0 0 0 0 0 -0.3" size="0.03" contype="0" conaffinity="0"/>',
                       '<geom type="capsule" fromto="0 0 0 0 0 -0.3" size="0.03" contype="0" conaffinity="0"/>'
                       '<site name="tip" pos="0 0 -0.3"/>').replace('<position joint="j0"', '<position name="a0" joint="j0"').replace(
  '</actuator></mujoco>', '''</actuator>
<sensor>
  <jointpos joint="j1"/> <jointvel joint="j2"/> <actuatorfrc actuator="a0"/>
  <accelerometer site="tip"/> <gyro site="tip"/> <velocimeter site="tip"/>
  <framepos objtype="site" objname="tip"/> <framequat objtype="site" objname="tip"/> <subtreecom body="world"/>
</sensor></mujoco>''')


@pytest.mark.gpu
def test_gpu_sparse_sensors_match_oracle():
  """Sensors on the sparse path (the sensor kernel runs after the sparse solve, mjw_step.hip run()):
  position, velocity and acceleration sensors of the chain against the oracle (no constraint rows, so
  qacc is the smooth solve and the acceleration sensors are held to the strict bar too)."""
  import torch

  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf
  from tests.test_gpu_parity_strict import normwise_close

  mjm = mjcf.load_model_from_string(SENSED.format(jac="sparse"))
  assert mjm.nsensor == 9
  nworld = 6
  rng = np.random.default_rng(4)
  qpos = rng.normal(0, 0.3, (nworld, mjm.nq))
  qvel = rng.normal(0, 2.0, (nworld, mjm.nv))
  ctrl = rng.uniform(-0.5, 0.5, (nworld, mjm.nu))
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=8, nconmax=4)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=8, nconmax=4)
  assert m.is_sparse
  mjw.forward(m, d)
  od.forward()
  torch.cuda.synchronize()
  normwise_close("sensordata", np_(d.sensordata), od.sensordata)
  m2, d2 = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=8, nconmax=4)
  mjw.step(m2, d2)
  od2 = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=8, nconmax=4)[1]
  od2.step()
  torch.cuda.synchronize()
  normwise_close("sensordata after step", np_(d2.sensordata), od2.sensordata)


@pytest.mark.gpu
@pytest.mark.parametrize("integrator", ["Euler", "implicitfast"])
def test_gpu_sparse_newton_humanoid_matches_oracle(integrator):
  """Newton on the sparse path (dense H = M + J'DJ per world, solver.py:2879-3008, as the reference
  builds for its sparse models): the humanoid forced onto the sparse path (jacobian="sparse") in
  contact, against the fp64 oracle at the solver bar (cost excess, qacc 5e-3), and one step."""
  import torch

  import mujoco_warp_amd as mjw
  from tests.common import humanoid_model, random_states
  from tests.parity_models import efc_cost
  from tests.test_gpu_parity_strict import normwise_close

  mjm = humanoid_model("NEWTON")
  mjw.override_model(mjm, ["opt.jacobian=sparse", f"opt.integrator={integrator}"])
  nworld = 16
  qpos, qvel, ctrl = random_states(mjm, nworld, seed=12)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl)
  assert m.is_sparse and m.sp_nH == mjm.nv
  for st in ("fwd_position", "fwd_velocity", "fwd_actuation", "fwd_acceleration"):
    getattr(mjw, st)(m, d)
    getattr(od, st)()
  mjw.solve(m, d)
  od.solve()
  torch.cuda.synchronize()
  nv = mjm.nv
  worst = 0.0
  for w in range(nworld):
    n = int(od.nefc[w, 0])
    assert n > 0 and int(d.nefc[w]) == n
    J = od.efc_J[w].reshape(od.njmax, nv)[:n]
    args = (J, od.efc_D[w, :n], od.efc_aref[w, :n], od.efc_type[w, :n], od.qM[w].reshape(nv, nv), od.qacc_smooth[w])
    c_or = efc_cost(*args, od.qacc[w], fl=od.efc_frictionloss[w, :n])
    c_gpu = efc_cost(*args, np_(d.qacc[w]), fl=od.efc_frictionloss[w, :n])
    worst = max(worst, (c_gpu - c_or) / abs(c_or))
  assert worst <= 1e-5, worst
  normwise_close("qacc", np_(d.qacc), od.qacc, tol=5e-3)
  assert int(np_(d.solver_niter).max()) <= 10  # Newton converges in a few iterations (CG takes tens)
  m2, d2 = gpu_from_state(mjm, qpos, qvel, ctrl)
  od2 = oracle_from_state(mjm, qpos, qvel, ctrl)[1]
  mjw.step(m2, d2)
  od2.step()
  torch.cuda.synchronize()
  normwise_close("qpos", np_(d2.qpos), od2.qpos)
  normwise_close("qvel", np_(d2.qvel), od2.qvel, tol=5e-3)
