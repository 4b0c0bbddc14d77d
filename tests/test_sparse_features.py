"""The dense feature set on the sparse / flex path (csrc/mjw_sparse.hip): connect / weld equality rows
(constraint.py:124-365, 792-1110), ball-joint limits (:1421-1543) and the RK4 integrator
(forward.py:357-491), which the sparse models run through the same rk4_kernel state bookkeeping as
the dense ones.

tests/test_equality.py's model (connect to the world and site to site, welds body / body and to the
world with torquescale, a limited ball joint, a joint equality; a plane for contacts) forced onto the
sparse path with jacobian="sparse": the equality and limit rows, which precede the contact rows, in
the reference's order against the fp64 oracle; forces, sensors and a rollout at the bars of the dense
test; RK4 rollouts against the oracle."""

import numpy as np
import pytest

from tests.common import assert_close, dense_efc_J, gpu_from_state, np_, oracle_from_state
from tests.test_equality import EQ_XML, _states

SPARSE_XML = EQ_XML.replace('<option timestep="0.002"/>', '<option timestep="0.002" jacobian="sparse" integrator="{integ}"/>')


def _model(integ="Euler"):
  from mujoco_warp_amd import mjcf

  return mjcf.load_model_from_string(SPARSE_XML.format(integ=integ))


def test_put_model_accepts_sparse_connect_weld_ball_rk4():
  import mujoco_warp_amd as mjw

  for integ in ("Euler", "RK4"):
    m = mjw.put_model(_model(integ), device="cpu")
    assert m.is_sparse and m.nlimited_ball == 1 and m.neq_cw == 4


@pytest.mark.gpu
def test_gpu_sparse_equality_ball_rows_match_oracle():
  import torch

  import mujoco_warp_amd as mjw

  mjm = _model()
  nworld = 32
  qpos, qvel, ctrl = _states(mjm, nworld, seed=5)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=64, nconmax=16)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=64, nconmax=16)
  assert m.is_sparse
  mjw.forward(m, d)
  od.forward()
  torch.cuda.synchronize()
  nv = mjm.nv
  for w in range(nworld):
    ne, nf, nl = int(od.ne[w, 0]), int(od.nf[w, 0]), int(od.nl[w, 0])
    assert (int(d.ne[w]), int(d.nf[w]), int(d.nl[w])) == (ne, nf, nl)
    assert int(d.nefc[w]) == int(od.nefc[w, 0])
    n = ne + nf + nl  # rows before the contacts: deterministic order on both sides
    np.testing.assert_array_equal(d.efc.type[w, :n].cpu().numpy(), od.efc_type[w, :n])
    np.testing.assert_array_equal(d.efc.id[w, :n].cpu().numpy(), od.efc_id[w, :n])
    assert_close(f"J[w{w}]", dense_efc_J(m, d, w)[:n], od.efc_J[w].reshape(od.njmax, nv)[:n], rtol=1e-4, atol=2e-5)
    for f in ("pos", "vel", "aref", "D"):
      assert_close(f"{f}[w{w}]", np_(getattr(d.efc, f)[w, :n]), getattr(od, "efc_" + f)[w, :n], rtol=1e-3, atol=1e-4)
  assert (od.nl[:, 0] > 0).any()  # some worlds start beyond the ball limit
  assert_close("qacc", np_(d.qacc), od.qacc, rtol=5e-3, atol=5e-2)
  assert_close("sensordata", np_(d.sensordata), od.sensordata, rtol=5e-3, atol=5e-2)
  m2, d2 = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=64, nconmax=16)
  om2, od2 = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=64, nconmax=16)
  for _ in range(10):
    mjw.step(m2, d2)
    od2.step()
  torch.cuda.synchronize()
  assert_close("qpos", np_(d2.qpos), od2.qpos, rtol=2e-3, atol=2e-3)
  assert_close("qvel", np_(d2.qvel), od2.qvel, rtol=2e-2, atol=2e-2)


@pytest.mark.gpu
def test_gpu_sparse_rk4_matches_oracle_and_dense():
  import torch

  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf

  mjm = _model("RK4")
  nworld = 8
  qpos, qvel, ctrl = _states(mjm, nworld, seed=7)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=64, nconmax=16)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=64, nconmax=16)
  dense = mjcf.load_model_from_string(SPARSE_XML.format(integ="RK4").replace(' jacobian="sparse"', ' jacobian="dense"'))
  m3, d3 = gpu_from_state(dense, qpos, qvel, ctrl, njmax=64, nconmax=16)
  assert m.is_sparse and not m3.is_sparse
  for _ in range(5):
    mjw.step(m, d)
    mjw.step(m3, d3)
    od.step()
  torch.cuda.synchronize()
  assert_close("qpos", np_(d.qpos), od.qpos, rtol=2e-3, atol=2e-3)
  assert_close("qvel", np_(d.qvel), od.qvel, rtol=2e-2, atol=2e-2)
  assert_close("qpos sparse vs dense", np_(d.qpos), np_(d3.qpos), rtol=2e-3, atol=2e-3)
  np.testing.assert_allclose(np_(d.time), 5 * 0.002, rtol=1e-6)


# ---- elliptic cones on the sparse path (solve_kernel<3>) ------------------------------------------
def _elliptic_sparse_humanoid(solver):
  import mujoco_warp_amd as mjw
  from tests.test_elliptic import _elliptic_humanoid

  mjm = _elliptic_humanoid(solver)
  mjw.override_model(mjm, ["opt.jacobian=sparse"])
  return mjm


def test_put_model_accepts_sparse_elliptic():
  import mujoco_warp_amd as mjw

  for solver in ("CG", "NEWTON"):
    m = mjw.put_model(_elliptic_sparse_humanoid(solver), device="cpu")
    assert m.is_sparse and int(m.opt.cone) == 1


@pytest.mark.gpu
@pytest.mark.parametrize("solver", ["CG", "NEWTON"])
def test_gpu_sparse_elliptic_rows_and_solve(solver):
  """The humanoid forced sparse with elliptic cones: the same rows by type as the oracle (contact rows
  are matched by count and type: the sparse collision kernel fills the pool in its own order), the J of
  the rows before the contacts, and the device solve's fp64 cone-aware cost on the oracle's rows within
  the reference's 1.025x of the oracle optimum (solver_test.py:317); Newton qacc at the dense test's bar."""
  import torch

  import mujoco_warp_amd as mjw
  from tests.test_elliptic import _elliptic_cost

  nworld = 32
  mjm = _elliptic_sparse_humanoid(solver)
  qpos, qvel, ctrl = random_states_h(mjm, nworld, seed=80)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl)
  assert m.is_sparse
  mjw.forward(m, d)
  od.forward()
  torch.cuda.synchronize()
  nv = mjm.nv
  total_ell = 0
  for w in range(nworld):
    n = int(od.nefc[w, 0])
    assert int(d.nefc[w]) == n
    t = d.efc.type[w, :n].cpu().numpy()
    np.testing.assert_array_equal(np.sort(t), np.sort(od.efc_type[w, :n]))
    total_ell += int((t == 7).sum())
    if n == 0:
      continue
    nc0 = int(od.ne[w, 0] + od.nf[w, 0] + od.nl[w, 0])
    Jo = od.efc_J[w].reshape(od.njmax, nv)[:nc0]
    if nc0:
      np.testing.assert_allclose(dense_efc_J(m, d, w)[:nc0], Jo, rtol=1e-4, atol=1e-5 * max(1.0, np.abs(Jo).max()))
    c_or = _elliptic_cost(mjm, od, w, od.qacc[w])
    c_gpu = _elliptic_cost(mjm, od, w, np_(d.qacc[w]))
    qs = od.qacc_smooth[w]
    floor = 1e-9 * (1.0 + qs @ od.qM[w].reshape(nv, nv) @ qs)
    assert c_gpu <= c_or + 0.025 * abs(c_or) + floor, (w, c_gpu, c_or, floor)
    if solver == "NEWTON":
      np.testing.assert_allclose(np_(d.qacc[w]), od.qacc[w], rtol=0.1, atol=0.1)
  assert total_ell > 3 * nworld
  assert (np_(d.efc.state) == 4).any()  # some contacts in the cone (middle) zone


def random_states_h(mjm, nworld, seed):
  from tests.common import random_states

  return random_states(mjm, nworld, seed=seed)


@pytest.mark.gpu
def test_gpu_sparse_elliptic_rollout_and_sliding_box():
  """A 5-step elliptic Newton rollout of the sparse humanoid against the oracle (qpos 1e-3, as the dense
  test), and the sliding box on the sparse path: cone-state forces on the cone surface, deceleration mu g."""
  import torch

  import mujoco_warp_amd as mjw
  from tests.test_elliptic import _model as sphere_model

  mjm = _elliptic_sparse_humanoid("NEWTON")
  qpos, qvel, ctrl = random_states_h(mjm, 16, seed=81)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl)
  for _ in range(5):
    mjw.step(m, d)
    od.step()
  torch.cuda.synchronize()
  e = np.abs(np_(d.qpos) - od.qpos).max(axis=1) / np.abs(od.qpos).max(axis=1)
  assert e.max() < 1e-3, e.max()

  mu, g = 0.4, 9.81
  bm = sphere_model(opt='solver="CG" jacobian="sparse"', type="box", size="0.3 0.3 0.01", z=0.0099, mu=mu, condim=3)
  nworld = 4
  mb = mjw.put_model(bm, device="cuda")
  assert mb.is_sparse
  db = mjw.make_data(bm, nworld=nworld, nconmax=16, njmax=64, device="cuda", m=mb)
  for _ in range(300):
    mjw.step(mb, db)
  db.xfrc_applied[:, 1, 0] = 2 * mu * g
  for _ in range(100):
    mjw.step(mb, db)
  v0 = np_(db.qvel[:, 0])
  ncone = 0
  for _ in range(100):
    mjw.step(mb, db)
    torch.cuda.synchronize()
    nacon = int(db.nacon[0])
    for c in range(nacon):
      w = int(db.contact.worldid[c])
      adr = db.contact.efc_address[c, :3].cpu().numpy()
      if adr[0] < 0 or int(db.efc.state[w, adr[0]]) != 4:
        continue
      f = np_(db.efc.force[w, adr])
      np.testing.assert_allclose(np.hypot(f[1], f[2]), mu * f[0], rtol=2e-3)
      ncone += 1
  v1 = np_(db.qvel[:, 0])
  assert ncone > 50
  np.testing.assert_allclose((v1 - v0) / (100 * 0.002), mu * g, rtol=0.03)


# ---- Newton on flex models past nv = 256 (the dense H of solver.py:2879-3008, nv x nv per world) ------
BIG_CLOTH = """<mujoco><option timestep="0.002" solver="Newton" iterations="20"/><worldbody>
<geom type="plane" size="2 2 .1"/><geom type="sphere" size=".15" pos="0 0 .15"/>
<flexcomp name="c" type="grid" count="10 10 1" spacing=".05 .05 .05" pos="0 0 .32" mass=".2" radius=".005" dim="2">
<edge equality="true"/><contact condim="3"/></flexcomp></worldbody></mujoco>"""


def test_put_model_accepts_big_flex_newton():
  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf

  mjm = mjcf.load_model_from_string(BIG_CLOTH)
  m = mjw.put_model(mjm, device="cpu")
  assert m.is_sparse and mjm.nv == 300 and m.sp_nH == 300


@pytest.mark.gpu
def test_gpu_big_flex_newton_matches_oracle():
  """A 10 x 10 towel (nv = 300) draped on a sphere, solved with Newton on the device: the fp64 cost of the
  device qacc on the oracle's rows within the reference's 1.025x of the oracle optimum (solver_test.py:317),
  and a 3-step rollout at the solver bar."""
  import torch

  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf
  from tests.parity_models import efc_cost
  from tests.test_gpu_parity_strict import normwise_close

  mjm = mjcf.load_model_from_string(BIG_CLOTH)
  nworld = 2
  rng = np.random.default_rng(2)
  qpos = np.tile(mjm.qpos0, (nworld, 1)) + rng.normal(0, 0.002, (nworld, mjm.nq))
  qpos[:, 2::3] -= 0.03  # lower the towel into the sphere
  qvel = rng.normal(0, 0.05, (nworld, mjm.nv))
  ctrl = np.zeros((nworld, mjm.nu))
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=2048, nconmax=512)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=2048, nconmax=512)
  mjw.forward(m, d)
  od.forward()
  torch.cuda.synchronize()
  nv = mjm.nv
  for w in range(nworld):
    n = int(od.nefc[w, 0])
    assert n > 0 and int(d.nefc[w]) == n and int(od.ncon[w, 0]) > 0
    J = od.efc_J[w].reshape(od.njmax, nv)[:n]
    args = (J, od.efc_D[w, :n], od.efc_aref[w, :n], od.efc_type[w, :n], od.qM[w].reshape(nv, nv), od.qacc_smooth[w])
    c_or = efc_cost(*args, od.qacc[w], fl=od.efc_frictionloss[w, :n])
    c_gpu = efc_cost(*args, np_(d.qacc[w]), fl=od.efc_frictionloss[w, :n])
    assert c_gpu <= c_or + 0.025 * abs(c_or), (w, c_gpu, c_or)
  normwise_close("qacc", np_(d.qacc), od.qacc, tol=5e-3)
  m2, d2 = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=2048, nconmax=512)
  om2, od2 = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=2048, nconmax=512)
  for _ in range(3):
    mjw.step(m2, d2)
    od2.step()
  torch.cuda.synchronize()
  normwise_close("qpos", np_(d2.qpos), od2.qpos)
  normwise_close("qvel", np_(d2.qvel), od2.qvel, tol=5e-3)
