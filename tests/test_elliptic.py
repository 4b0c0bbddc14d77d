"""Elliptic friction cones (opt.cone = ELLIPTIC): contact rows
(constraint.py:1940-2200), the cone states of update_constraint (solver.py:1886-1942), the elliptic
line-search terms (solver.py:263-323, 1550-1611), the Newton cone Hessian (solver.py:2430-2585) and the
elliptic contact force (support.py:267-310).

The reference's elliptic tests compare against MuJoCo C at run time (no stored vectors), so the oracle
restatement is pinned here by analytic invariants: a resting sphere carries its weight with no friction
force, a sliding box's friction force lies on the cone surface (|f_t| = mu f_n) and decelerates it at
about mu g, a frictionless contact gives the pyramidal rows, CG and Newton reach the same optimum, and the
Newton solution is stationary.  `-m gpu` tests compare the HIP path with the oracle.
"""

import numpy as np
import pytest

from tests.common import gpu_from_state, humanoid_model, np_, oracle_from_state, random_states

SPHERE = """<mujoco><option timestep="0.002" cone="elliptic" {opt}/><worldbody><geom type="plane" size="5 5 .1" friction="{mu} 0.005 0.0001" condim="{condim}"/>
<body pos="0 0 {z}"><freejoint/><geom type="{type}" size="{size}" mass="{mass}" friction="{mu} 0.005 0.0001" condim="{condim}"/></body>
</worldbody></mujoco>"""


def _model(**kw):
  from mujoco_warp_amd import mjcf

  args = dict(opt='solver="Newton"', z=0.1, type="sphere", size="0.1", mass=1.0, mu=0.5, condim=3)
  args.update(kw)
  return mjcf.load_model_from_string(SPHERE.format(**args))


def _oracle(mjm, qpos, qvel, njmax=32, nconmax=8):
  from oracle import orc

  od = orc.OracleData(orc.OracleModel(mjm), qpos.shape[0], njmax, nconmax)
  od.qpos[:] = qpos
  od.qvel[:] = qvel
  return od


def _contact_force(od, w=0):
  """Contact-frame force of contact 0 of world w: elliptic rows are the force components."""
  n = int(od.ncon[w, 0])
  assert n >= 1
  dim = int(od.con_dim[w, 0])
  adr = od.con_efc_address[w, :dim]
  return od.efc_force[w, adr], dim


def test_oracle_resting_sphere_weight_no_friction():
  mjm = _model(z=0.0995)
  assert int(mjm.opt.cone) == 1
  od = _oracle(mjm, mjm.qpos0[None], np.zeros((1, 6)))
  for _ in range(500):
    od.step()
  od.forward()
  f, dim = _contact_force(od)
  assert dim == 3 and int(od.nefc[0, 0]) == 3
  assert list(od.efc_type[0, :3]) == [7, 7, 7]
  g = 9.81
  np.testing.assert_allclose(f[0], g * 1.0, rtol=2e-3)  # normal force = m g
  assert np.abs(f[1:]).max() < 1e-6 * g
  assert np.abs(od.qvel[0]).max() < 1e-4


def test_oracle_sliding_box_on_the_cone_surface():
  """A flat box pushed sideways by 2 mu m g slides: its friction force lies on the cone surface,
  |f_t| = mu f_n, opposes the motion, and the box accelerates at (F - mu m g) / m = mu g."""
  mu, g = 0.4, 9.81
  mjm = _model(type="box", size="0.3 0.3 0.01", z=0.0099, mu=mu, condim=3)  # flat: no tipping
  od = _oracle(mjm, mjm.qpos0[None], np.zeros((1, 6)), njmax=64, nconmax=16)
  for _ in range(300):  # settle on the plane first
    od.step()
  od.xfrc_applied[0, 6] = 2 * mu * g  # body 1, force x (mass 1)
  for _ in range(100):
    od.step()
  v0 = od.qvel[0, 0]
  n = 100
  ncone = 0
  for _ in range(n):
    od.step()
    # the soft contacts of the sliding box chatter (corner contacts come and go), but every contact in
    # the cone (middle) zone has its force exactly on the cone surface, opposing the motion
    for c in range(int(od.ncon[0, 0])):
      adr = od.con_efc_address[0, 10 * c: 10 * c + 3]
      if adr[0] < 0 or od.efc_state[0, adr[0]] != 4:
        continue
      assert (od.efc_state[0, adr] == 4).all()
      f = od.efc_force[0, adr]
      np.testing.assert_allclose(np.hypot(f[1], f[2]), mu * f[0], rtol=1e-9)
      assert f[1] * od.con_frame[0, 9 * c + 3] + f[2] * od.con_frame[0, 9 * c + 6] < 0
      ncone += 1
  v1 = od.qvel[0, 0]
  assert v0 > 0.1 and ncone > 50
  np.testing.assert_allclose((v1 - v0) / (n * 0.002), mu * g, rtol=0.02)


def test_oracle_condim1_elliptic_equals_pyramidal():
  """A frictionless contact has one row either way; the cone choice must not change it."""
  from mujoco_warp_amd import mjcf

  xml = SPHERE.format(opt='solver="Newton"', z=0.0995, type="sphere", size="0.1", mass=1.0, mu=0.5, condim=1)
  me = mjcf.load_model_from_string(xml)
  mp = mjcf.load_model_from_string(xml.replace('cone="elliptic"', 'cone="pyramidal"'))
  qvel = np.array([[0.3, -0.2, -0.5, 0.1, 0.2, 0.0]])
  a, b = _oracle(me, me.qpos0[None], qvel), _oracle(mp, mp.qpos0[None], qvel)
  for _ in range(5):
    a.step()
    b.step()
  np.testing.assert_array_equal(a.qpos, b.qpos)
  np.testing.assert_array_equal(a.efc_type[:, :1], b.efc_type[:, :1])


def _elliptic_humanoid(solver, iterations=None):
  mjm = humanoid_model(solver, iterations=iterations)
  mjm.opt.cone = 1
  return mjm


def test_oracle_elliptic_cg_and_newton_reach_the_same_optimum():
  nworld = 8
  mc, mn = _elliptic_humanoid("CG", iterations=500), _elliptic_humanoid("NEWTON", iterations=100)
  mc.opt.tolerance = mn.opt.tolerance = 1e-12
  qpos, qvel, ctrl = random_states(mc, nworld, seed=3)
  _, oc = oracle_from_state(mc, qpos, qvel, ctrl)
  _, on = oracle_from_state(mn, qpos, qvel, ctrl)
  oc.forward()
  on.forward()
  nefc = oc.nefc[:, 0]
  assert (nefc == on.nefc[:, 0]).all() and nefc.sum() > 5 * nworld
  assert (oc.efc_type == 7).any()
  cost_c, cost_n = oc.solver_cost[:, 0], on.solver_cost[:, 0]
  np.testing.assert_allclose(cost_c, cost_n, rtol=1e-6, atol=1e-9)
  err = np.abs(oc.qacc - on.qacc).max(axis=1) / (np.abs(on.qacc).max(axis=1) + 1)
  assert err.max() < 1e-3
  # some contacts actually sit in the cone (middle) zone
  assert (on.efc_state == 4).any()


def test_oracle_elliptic_newton_is_stationary():
  """At the Newton solution the cost gradient M (qacc - qacc_smooth) - J' f vanishes."""
  nworld = 8
  mjm = _elliptic_humanoid("NEWTON", iterations=100)
  mjm.opt.tolerance = 1e-12
  qpos, qvel, ctrl = random_states(mjm, nworld, seed=4)
  _, od = oracle_from_state(mjm, qpos, qvel, ctrl)
  od.forward()
  nv = mjm.nv
  for w in range(nworld):
    n = int(od.nefc[w, 0])
    M = od.qM[w].reshape(nv, nv)
    J = od.efc_J[w].reshape(od.njmax, nv)[:n]
    g = M @ (od.qacc[w] - od.qacc_smooth[w]) - J.T @ od.efc_force[w, :n]
    assert np.abs(g).max() < 1e-6 * (1 + np.abs(od.qfrc_smooth[w]).max()), (w, np.abs(g).max())


def test_contact_force_elliptic_rows_are_the_force(tmp_path):
  """support.contact_force with elliptic cones returns the contact's rows directly (support.py:296-299)."""
  import torch

  import mujoco_warp_amd as mjw

  mjm = _model()
  m = mjw.put_model(mjm, device="cpu")
  d = mjw.make_data(mjm, nworld=2, nconmax=4, njmax=16, device="cpu", m=m)
  d.nacon[0] = 2
  d.contact.dim[:2] = torch.tensor([3, 3], dtype=torch.int32)
  d.contact.worldid[:2] = torch.tensor([0, 1], dtype=torch.int32)
  d.contact.efc_address[0, :3] = torch.tensor([0, 1, 2], dtype=torch.int32)
  d.contact.efc_address[1, :3] = torch.tensor([3, 4, 5], dtype=torch.int32)
  d.contact.frame[:2] = torch.eye(3)
  d.efc.force[0, :3] = torch.tensor([5.0, 1.0, -2.0])
  d.efc.force[1, 3:6] = torch.tensor([7.0, 0.5, 0.25])
  out = torch.zeros((2, 6))
  mjw.contact_force(m, d, torch.tensor([0, 1]), False, out)
  np.testing.assert_array_equal(out.numpy(), [[5, 1, -2, 0, 0, 0], [7, 0.5, 0.25, 0, 0, 0]])


# ---- GPU ------------------------------------------------------------------------------------------
def _gpu_pair(solver, nworld, seed, njmax=64):
  mjm = _elliptic_humanoid(solver)
  qpos, qvel, ctrl = random_states(mjm, nworld, seed=seed)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=njmax)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=njmax)
  return mjm, m, d, od


@pytest.mark.gpu
@pytest.mark.parametrize("njmax", [64, 128])
@pytest.mark.parametrize("solver", ["CG", "NEWTON"])
def test_gpu_elliptic_rows_and_solve(solver, njmax):
  """Elliptic rows (same count / order / type, J and scalars) and the device solve: fp64 cost within the
  reference's 1.025x of the oracle optimum (solver_test.py:317); Newton qacc at the reference's
  solver bar (solver_test.py:32-38: 5e-3 * 20).  njmax 64: the register-resident dense solve; njmax 128:
  the generic LDS solver (rows past one wavefront, the cone at the first row of each contact)."""
  import torch

  import mujoco_warp_amd as mjw

  nworld = 32
  mjm, m, d, od = _gpu_pair(solver, nworld, seed=80, njmax=njmax)
  mjw.forward(m, d)
  od.forward()
  torch.cuda.synchronize()
  nv = mjm.nv
  total_ell = 0
  for w in range(nworld):
    n = int(od.nefc[w, 0])
    assert int(d.nefc[w]) == n
    t = d.efc.type[w, :n].cpu().numpy()
    np.testing.assert_array_equal(t, od.efc_type[w, :n])
    total_ell += int((t == 7).sum())
    if n == 0:
      continue
    Jg = np_(d.efc.J[w, :n, :nv])
    Jo = od.efc_J[w].reshape(od.njmax, nv)[:n]
    np.testing.assert_allclose(Jg, Jo, rtol=1e-4, atol=1e-5 * np.abs(Jo).max())
    np.testing.assert_allclose(np_(d.efc.D[w, :n]), od.efc_D[w, :n], rtol=3e-4)
    np.testing.assert_allclose(np_(d.efc.aref[w, :n]), od.efc_aref[w, :n], rtol=3e-4, atol=1e-3 * (np.abs(od.efc_aref[w, :n]).max() + 1))
    # cone-aware fp64 cost on the oracle's rows, at the oracle optimum and at the device solution
    c_or = _elliptic_cost(mjm, od, w, od.qacc[w])
    np.testing.assert_allclose(c_or, od.solver_cost[w, 0], rtol=1e-9, atol=1e-12)
    c_gpu = _elliptic_cost(mjm, od, w, np_(d.qacc[w]))
    # absolute floor: fp32 round-off of an unconstrained solve, 0.5 e' M e with |e| ~ 1e-6 |qacc_smooth|
    qs = od.qacc_smooth[w]
    floor = 1e-9 * (1.0 + qs @ od.qM[w].reshape(nv, nv) @ qs)
    assert c_gpu <= c_or + 0.025 * abs(c_or) + floor, (w, c_gpu, c_or, floor)
    if solver == "NEWTON":
      np.testing.assert_allclose(np_(d.qacc[w]), od.qacc[w], rtol=0.1, atol=0.1)
  assert total_ell > 3 * nworld


def _elliptic_cost(mjm, od, w, qacc):
  """fp64 primal cost of qacc on the oracle's rows with elliptic cones (solver.py:1886-1942 costs)."""
  nv = mjm.nv
  n = int(od.nefc[w, 0])
  J = od.efc_J[w].reshape(od.njmax, nv)[:n]
  M = od.qM[w].reshape(nv, nv)
  dq = qacc - od.qacc_smooth[w]
  c = 0.5 * dq @ M @ dq
  jar = J @ qacc - od.efc_aref[w, :n]
  D = od.efc_D[w, :n]
  ne, nf = int(od.ne[w, 0]), int(od.nf[w, 0])
  iri = 1.0 / np.sqrt(max(mjm.opt.impratio, 1e-15))
  for r in range(n):
    t = od.efc_type[w, r]
    if r < ne:
      c += 0.5 * D[r] * jar[r] ** 2
    elif r < ne + nf:
      f = od.efc_frictionloss[w, r]
      rf = f / D[r]
      c += -f * (0.5 * rf + jar[r]) if jar[r] <= -rf else (-f * (0.5 * rf - jar[r]) if jar[r] >= rf else 0.5 * D[r] * jar[r] ** 2)
    elif t != 7:
      c += 0.5 * D[r] * jar[r] ** 2 if jar[r] < 0 else 0.0
    else:
      con = od.efc_id[w, r]
      adr = od.con_efc_address[w, 10 * con: 10 * con + 10]
      if adr[0] != r:
        continue
      dim = int(od.con_dim[w, con])
      fr = od.con_friction[w, 5 * con: 5 * con + 5]
      mu = fr[0] * iri
      N = jar[r] * mu
      u = np.array([jar[adr[j]] * fr[j - 1] for j in range(1, dim)])
      T = np.sqrt((u * u).sum())
      if N >= mu * T:
        continue
      if mu * N + T <= 0:
        c += sum(0.5 * D[adr[j]] * jar[adr[j]] ** 2 for j in range(dim))
      else:
        dm = D[r] / (mu * mu * (1 + mu * mu))
        c += 0.5 * dm * (N - mu * T) ** 2
  return c


@pytest.mark.gpu
def test_gpu_elliptic_step_rollout_and_sliding_box():
  """A 5-step elliptic Newton rollout against the oracle (normwise qpos 1e-3), and the device sliding
  box: every cone-state contact force on the cone surface, acceleration mu g."""
  import torch

  import mujoco_warp_amd as mjw

  for njmax in (64, 128):  # register-resident and generic solves
    mjm, m, d, od = _gpu_pair("NEWTON", 16, seed=81, njmax=njmax)
    for _ in range(5):
      mjw.step(m, d)
      od.step()
    torch.cuda.synchronize()
    e = np.abs(np_(d.qpos) - od.qpos).max(axis=1) / np.abs(od.qpos).max(axis=1)
    assert e.max() < 1e-3, (njmax, e.max())

  mu, g = 0.4, 9.81
  bm = _model(type="box", size="0.3 0.3 0.01", z=0.0099, mu=mu, condim=3)
  nworld = 4
  mb = mjw.put_model(bm, device="cuda")
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
